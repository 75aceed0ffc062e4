# FETCH_SIZE and WRITE_SIZE (one pass each) over c4 --device-encode at 262,144
# txs: the Kryo encoder kernels' L2-to-fabric bytes, for the devenc bench line's
# traffic (tools/pmc_kryo_traffic.py composes profiles/r04_pmc_kryo_traffic.json)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_kryo2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --workload c4 --device-encode --c4-txs 262144 --steps 1 --warmup 0 --no-cpu-baseline --no-clock"
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmck_$i -o p -- $BENCH > $O/pass$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
  find /tmp/pmck_$i -name "*counter_collection.csv" -exec cp {} $O/pass$i.csv \;
done
python3 $R/tools/pmc_summary.py --all $O/pass*.csv > $O/summary.json && python3 -c "
import json; s=json.load(open('$O/summary.json'))
for k,v in s.items():
    if 'kryo' in k or 'Scan' in k or 'scan' in k: print(k[:80], v)"
