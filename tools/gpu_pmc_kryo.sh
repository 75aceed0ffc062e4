# One rocprofv3 counter pass over c4 --device-encode (262,144 txs): instruction
# mix and wait cycles of the Kryo encoder kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_kryo
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d /tmp/pmck -o p -- python3 $R/bench.py --workload c4 --device-encode --c4-txs 262144 --steps 1 --warmup 0 --no-cpu-baseline --no-clock > $O/pass.log 2>&1 || { echo "pmc failed"; tail -5 $O/pass.log; exit 1; }
find /tmp/pmck -name "*counter_collection.csv" -exec cp {} $O/pass.csv \;
python3 - <<PY
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); calls = collections.Counter()
for r in csv.DictReader(open("$O/pass.csv")):
    n = r["Kernel_Name"]
    if "kryo" not in n: continue
    agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, c in agg.items(): print(n[:60], dict(c))
PY
