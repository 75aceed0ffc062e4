# r05: GPU Kryo encoder iteration -- parity tests, the encoder alone, its kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kryo.py tests/test_gpu_txcomp.py > $O/pytest_kryo.log 2>&1 || { echo "kryo tests failed"; tail -30 $O/pytest_kryo.log; exit 1; }
tail -2 $O/pytest_kryo.log
timeout -k 10 300 python -u tools/kryo_dev_bench.py > $O/kbench.json 2> $O/kbench.err || { echo "kbench failed"; tail -20 $O/kbench.err; exit 1; }
cat $O/kbench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p5b -o kb -- python3 $R/tools/kryo_dev_bench.py --calls 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
find /tmp/p5b -name "*kernel_stats.csv" -exec cp {} $O/kb_kernel_stats.csv \;
python3 - <<PY
import csv
r=list(csv.DictReader(open("$O/kb_kernel_stats.csv")))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:12]: print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us')
PY
