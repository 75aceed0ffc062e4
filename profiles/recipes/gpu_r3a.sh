# round 3 first call: GPU suite, then C2 and C3 bench lines with the open-lane oracle checks
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for wl in c2 c3; do
  timeout -k 10 400 python -u bench.py --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo "bench $wl failed"; tail -20 $O/bench_$wl.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$wl.json'));print('$wl', round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],2), 'ms', d['verdict_check'], d['cpu_baseline'])"
done
