# r06: device paths with the id chain forked beside the prep key half -- A/B CORDAHIP_DEVICE_SPLIT on c4 and c4 --device-encode
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6i
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_txcomp.py tests/test_gpu_runtime.py -k "not 2_29" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name, args
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 10 --warmup 2 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k})"
}
for k in 1 2; do
  CORDAHIP_DEVICE_SPLIT=0 run c4_nosplit$k "--workload c4" && run c4_split$k "--workload c4" && \
  CORDAHIP_DEVICE_SPLIT=0 run c4de_nosplit$k "--workload c4 --device-encode" && run c4de_split$k "--workload c4 --device-encode" || exit 1
done
