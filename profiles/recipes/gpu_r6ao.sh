# r06: the host calls' templates-only chain as one fused shape + hash launch per id
# slice (CORDAHIP_KRYO_FUSED=1) against kryo_shape + kryo_hash: the component tests
# with the fused kernel, then c4h --components --inflight 2 alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6ao}
mkdir -p $O
cd $R
CORDAHIP_KRYO_FUSED=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_txcomp.py tests/test_gpu_kryo_fuzz.py tests/test_gpu_memory.py -x -q --timeout 300 --timeout-method thread -k "not 2_29" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 20 --warmup 4 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
HC="--workload c4h --components --inflight 2"
for rep in ${REPS:-1 2 3}; do
  run base_$rep "$HC" && CORDAHIP_KRYO_FUSED=1 run fused_$rep "$HC" || exit 1
done
