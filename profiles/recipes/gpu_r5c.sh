# r05: PMC passes over the GPU Kryo encoder alone (tools/kryo_dev_bench.py, 262,144 txs, 2 calls)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/tools/kryo_dev_bench.py --txs 262144 --calls 2"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TCC_WRITE_REQ TCP_TCC_READ_REQ"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc5c_$i -o p -- $B > $O/pass$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
  find /tmp/pmc5c_$i -name "*counter_collection.csv" -exec cp {} $O/pass$i.csv \;
done
python3 $R/tools/pmc_summary.py $O/pass*.csv > $O/summary.json && python3 -c "
import json; s=json.load(open('$O/summary.json'))
for k,v in s.items():
    if 'kryo' in k: print(k[:60], {a: round(b) for a,b in v.items()})"
