# r06: overlapped signed-tx calls -- the tx GPU tests, then c4 / c4h / c4h --components
# at --inflight 1 and 2 on one box, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_txcomp.py tests/test_gpu_tx.py tests/test_gpu_runtime.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
run() {  # name, args
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 10 --warmup 2 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k})"
}
run c4 "--workload c4" && run c4h1 "--workload c4h" && run c4h2 "--workload c4h --inflight 2" && \
run c4hc1 "--workload c4h --components" && run c4hc2 "--workload c4h --components --inflight 2" && \
run c4b "--workload c4" && run c4h2b "--workload c4h --inflight 2" && run c4hc2b "--workload c4h --components --inflight 2"
