# r06: the device component call -- txcomp / tx / kryo GPU tests, then c4, c4 --device-encode, c4h --components --inflight 2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6c
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_txcomp.py -k 2_29 -x -v -s --timeout 380 --timeout-method thread 2>&1 | tee $O/pytest_big.log || { echo "big test failed"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_txcomp.py tests/test_gpu_tx.py tests/test_gpu_kryo.py tests/test_gpu_kryo_fuzz.py -k "not 2_29" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
run() {  # name, args
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 10 --warmup 2 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k})"
}
run c4 "--workload c4" && run c4de "--workload c4 --device-encode" && run c4hc2 "--workload c4h --components --inflight 2" && run c4de2 "--workload c4 --device-encode"
