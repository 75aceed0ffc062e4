# r06: the device hash chain's fused steady state (one shape + hash launch, misses to
# the direct encoder; CORDAHIP_KRYO_DEVICE_FUSED=0: the full chain every call): the
# device-path tests, then C4 --device-encode alternating (rocprofv3 kernel stats)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ar
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_txcomp.py tests/test_gpu_device_chunks.py tests/test_gpu_kryo.py tests/test_gpu_kryo_fuzz.py tests/test_gpu_memory.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 10 --warmup 2 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
DE="--workload c4 --device-encode"
for rep in 1 2 3; do
  run fused_$rep "$DE" && CORDAHIP_KRYO_DEVICE_FUSED=0 run full_$rep "$DE" || exit 1
done
