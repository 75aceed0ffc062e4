# host-pipeline bench lines with traces (WLS), then a slice of the fully oracle-checked agreement sweep
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r3e}
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for wl in ${WLS:-c2h c3h c4h}; do
  CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$wl.json 2> $O/trace_$wl.err || { echo "bench $wl failed"; tail -5 $O/trace_$wl.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$wl.json'));print('$wl', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', d['verdict_check'].get('mismatches_vs_construction'), d['verdict_check'].get('mismatches_vs_oracle_open_lanes'))"
  grep "cordahip" $O/trace_$wl.err | tail -8
done
if [ -n "$ED$EC" ]; then
  timeout -k 10 ${SWEEP_S:-900} python -u tools/agree_1e9.py --oracle-all --ed ${ED:-0} --ec ${EC:-0} --first ${FIRST:-0} --threads 16 --log $O/agree_log.jsonl > $O/agree.out 2>&1; rc=$?
  tail -3 $O/agree.out
  exit $rc
fi
