# signed-tx boundary after the id-copy stream and slice-sized signature chunks:
# GPU tx/multi-device/host-batch tests, then c4h x3, c2h, c3h, c5 (no CPU baseline)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3m
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_multidevice.py tests/test_gpu_host_batch.py tests/test_gpu_stream.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for wl in ${WLS:-c4h c4h c4h c2h c3h c5}; do
  i=$((i+1))
  CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_${wl}_$i.json 2> $O/trace_${wl}_$i.err || { echo "bench $wl failed"; tail -n 5 $O/trace_${wl}_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_${wl}_$i.json'));print('$wl', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', d['verdict_check'].get('mismatches_vs_construction'), d['verdict_check'].get('mismatches_vs_oracle_open_lanes'))"
done
