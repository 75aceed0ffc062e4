# Round measurement pass (run through gpurun): the full GPU test suite, then
# the bench line of every workload (default steps/warmup, CPU baseline on).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for wl in ${WLS:-c2 c3 c1 c4 c5}; do
  timeout -k 10 600 python -u bench.py --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo "bench $wl failed"; tail -20 $O/bench_$wl.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$wl.json'));print('$wl', round(d['value']/1e6,2), 'M/s', d['verdict_check'])"
done
