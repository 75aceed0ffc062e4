# r05: GPU Kryo template encoder -- parity, then the device-encode C4 line and its kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5a
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kryo.py tests/test_gpu_txcomp.py > $O/pytest_kryo.log 2>&1 || { echo "kryo tests failed"; tail -30 $O/pytest_kryo.log; exit 1; }
tail -3 $O/pytest_kryo.log
timeout -k 10 400 python -u bench.py --workload c4 --device-encode --steps 5 --warmup 1 --no-cpu-baseline > $O/c4de.json 2> $O/c4de.err || { echo "bench failed"; tail -20 $O/c4de.err; exit 1; }
cat $O/c4de.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p5a -o c4de -- python3 $R/bench.py --workload c4 --device-encode --steps 2 --warmup 1 --no-cpu-baseline --no-clock > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
find /tmp/p5a -name "*kernel_stats.csv" -exec cp {} $O/c4de_kernel_stats.csv \;
python3 - <<PY
import csv
r=list(csv.DictReader(open("$O/c4de_kernel_stats.csv")))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:14]: print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e6,3), x['Percentage'])
PY
cd $R
timeout -k 10 300 python3 tools/microbench/radix32_ab.py 256 $O/r05_radix32_ab.json > $O/radix32.log 2>&1 || { echo "radix32 failed"; tail -20 $O/radix32.log; exit 1; }
cat $O/radix32.log
