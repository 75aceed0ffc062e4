# Round-4 GPU call: optional GPU suite + smoke, bench lines (roofline, cpu_baseline,
# clock under load), rocprofv3 kernel stats. TAG names gpurun_out/r4_$TAG;
# TESTS=1 runs the suite first; WLS lists bench workloads; PROF lists rocprof ones.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_${TAG:-x}
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest.log; exit 1; }
  tail -n 1 $O/pytest.log
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -n 10 $O/smoke.log; exit 1; }
  tail -n 1 $O/smoke.log
fi
# WLS entries: workload[:extra+args] (e.g. c4h:--native-leaves)
for spec in $WLS; do
  wl=${spec%%:*}
  extra=""
  [ "$spec" != "$wl" ] && extra=$(echo "${spec#*:}" | tr '+' ' ')
  tag=$(echo "$spec" | tr ':+' '__' | tr -d '-')
  timeout -k 10 420 python -u bench.py --workload $wl $extra $BENCH_ARGS > $O/bench_$tag.json 2> $O/bench_$tag.err || { echo "bench $spec failed"; tail -20 $O/bench_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$tag.json'));c=d['verdict_check'];print('$tag', round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],2), 'ms frac', round(d['roofline']['frac'],3), 'clk', d.get('clock_ghz'), 'v/Mclk', round(d.get('verifs_per_mclk') or 0), 'mism', c.get('mismatches_vs_construction'), c.get('mismatches_vs_oracle_open_lanes'), 'lanes', c.get('lanes_checked'), 'cpu', round((d.get('cpu_baseline') or {}).get('value') or 0))"
done
for wl in $PROF; do
  TAG=r4${TAG}_$wl WL=$wl bash tools/gpu_prof.sh > $O/prof_$wl.txt || { echo "prof $wl failed"; tail -5 $O/prof_$wl.txt; exit 1; }
  cp gpurun_out/prof/r4${TAG}_${wl}_kernel_stats.csv $O/
  head -6 $O/prof_$wl.txt
done
