# Round-3 re-entry check: full GPU suite, smoke, default bench (C2), then the
# boundary lines c2h / c4h with host traces
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r3h}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -n 10 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 failed"; tail -n 5 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
for WL in ${WLS:-c2h c4h}; do
  CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$WL.json 2> $O/trace_$WL.err || { echo "bench $WL failed"; tail -n 5 $O/trace_$WL.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$WL.json'));print('$WL', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', d['verdict_check'].get('mismatches_vs_construction'), d['verdict_check'].get('mismatches_vs_oracle_open_lanes'))"
done
