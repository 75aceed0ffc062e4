# r06: device signed-tx calls with the Ed25519 section in alternating 2^k-signature
# chunks (CORDAHIP_DEVICE_ED_CHUNK; 0 = one launch pair) -- device-path tests, then
# c4 and c4 --device-encode A/B, alternating, one box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6t
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_txcomp.py tests/test_gpu_runtime.py tests/test_gpu_memory.py -x -q --timeout 300 --timeout-method thread -k "not 2_29" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 10 --warmup 2 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
for rep in 1 2; do
  CORDAHIP_DEVICE_ED_CHUNK=0 run c4_c0_$rep "--workload c4" && CORDAHIP_DEVICE_ED_CHUNK=131072 run c4_c17_$rep "--workload c4" && \
  CORDAHIP_DEVICE_ED_CHUNK=262144 run c4_c18_$rep "--workload c4" && CORDAHIP_DEVICE_ED_CHUNK=65536 run c4_c16_$rep "--workload c4" && \
  CORDAHIP_DEVICE_ED_CHUNK=0 run de_c0_$rep "--workload c4 --device-encode" && CORDAHIP_DEVICE_ED_CHUNK=131072 run de_c17_$rep "--workload c4 --device-encode" && \
  CORDAHIP_DEVICE_ED_CHUNK=262144 run de_c18_$rep "--workload c4 --device-encode" || exit 1
done
