# Round-4 GPU call o: chunk-aligned id slices -- tx tests, c4h chunk x lookahead
# grid beside C4, then one host-traced c4h run (CORDAHIP_TRACE)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_${TAG:-o}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_multidevice.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
run() {  # name, env, workload
  env $2 timeout -k 10 300 python -u bench.py --workload $3 --steps 5 --warmup 1 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$1.json'));c=d['verdict_check'];print('$1', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms clk', round(d.get('clock_ghz') or 0,3), 'mism', c.get('mismatches_vs_construction'), c.get('txid_mismatches_vs_device_path'))"
}
for c in 65536 131072; do for a in 1 2; do run c4h_${c}_a$a "CORDAHIP_TX_SIG_CHUNK=$c CORDAHIP_TX_SLICE_AHEAD=$a" c4h || exit 1; done; done
run c4 X=1 c4 || exit 1
CORDAHIP_TRACE=1 CORDAHIP_TX_SIG_CHUNK=65536 timeout -k 10 300 python -u bench.py --workload c4h --steps 3 --warmup 1 --no-cpu-baseline --no-clock > $O/c4h_traced.json 2> $O/c4h_traced.err || { echo "traced failed"; exit 1; }
grep "signed tx batch" $O/c4h_traced.err | tail -3
