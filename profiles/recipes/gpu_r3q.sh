# two Ed25519 streams/workspaces in the packed host pipeline (CORDAHIP_ED_STREAMS 2 vs 1)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3q
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_multidevice.py tests/test_gpu_host_batch.py tests/test_gpu_ed25519.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for v in 2 1 2 1; do
  for wl in c4h c2h; do
    CORDAHIP_ED_STREAMS=$v timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_${wl}_$v.json 2> $O/err_${wl}_$v.err || { echo "bench $wl $v failed"; tail -n 5 $O/err_${wl}_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${wl}_$v.json'));print('$wl ed_streams $v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', d['verdict_check'].get('mismatches_vs_construction'), d['verdict_check'].get('mismatches_vs_oracle_open_lanes'))"
  done
done
