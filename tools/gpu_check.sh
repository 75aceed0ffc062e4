# Full GPU check: the -m gpu suite, then bench lines for the given workloads
# (WLS, default "c3 c2"), then a rocprofv3 kernel-stats pass of PROF (default c3).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/check
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for wl in ${WLS:-c3 c2}; do
  timeout -k 10 600 python bench.py --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo "bench $wl failed"; tail -20 $O/bench_$wl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$wl.json')); print('$wl', round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],1), 'ms', round(d['roofline']['frac'],3), d['verdict_check'], d.get('cpu_baseline',{}).get('gpu_vs_port_mismatches_on_sample'))"
done
if [ -n "${PROF:-c3}" ]; then TAG=${TAG:-prof_${PROF:-c3}} WL=${PROF:-c3} bash tools/gpu_prof.sh; fi
