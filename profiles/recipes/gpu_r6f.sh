# r06: SQ counters of the device component chain's kernels (c4 --device-encode, 262,144 txs)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export CORDAHIP_KRYO_HASH_WAVES=${W:-5}
BENCH="python3 $R/bench.py --workload c4 --device-encode --c4-txs 262144 --steps 2 --warmup 1 --no-cpu-baseline --no-clock"
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc_1 -o p -- $BENCH > $O/pass1.log 2>&1 || { echo "pmc pass failed"; tail -5 $O/pass1.log; exit 1; }
find /tmp/pmc_1 -name "*counter_collection.csv" -exec cp {} $O/pass1.csv \;
python3 $R/tools/pmc_summary.py $O/pass1.csv > $O/summary.json && python3 -c "
import json; s=json.load(open('$O/summary.json'))
for k,v in s.items():
    if 'kryo' in k or 'merkle' in k or 'sha256' in k: print(k[-40:], {a: round(b) for a,b in v.items()})"
