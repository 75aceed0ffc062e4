# r06: ECDSA chunks of the host pipelines alternating over two workspaces / streams
# (s_ec + slot 0, s_ec2 + slot 1): the ECDSA-path GPU tests, then C3 / c3h / c3h
# --inflight 2 / C5, alternating on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6ai}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_ecdsa.py tests/test_gpu_host_batch.py tests/test_gpu_runtime.py tests/test_gpu_multidevice.py tests/test_gpu_csr.py tests/test_gpu_memory.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 5 --warmup 1 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), d.get('device_mem_gb', {}).get('peak'), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
for rep in 1 2; do
  run c3_$rep "--workload c3" && run c3h1_$rep "--workload c3h" && run c3h2_$rep "--workload c3h --inflight 2" && \
  run c5_$rep "--workload c5" || exit 1
done
