# signed-tx boundary (c4h): tx-id slice copies on their own stream; A/B of the
# signature chunk size; GPU tx tests first
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3k
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_multidevice.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for ch in ${CHUNKS:-524288 262144 131072}; do
  CORDAHIP_TX_SIG_CHUNK=$ch CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload c4h --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4h_$ch.json 2> $O/trace_c4h_$ch.err || { echo "bench $ch failed"; tail -n 5 $O/trace_c4h_$ch.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c4h_$ch.json'));print('c4h chunk $ch', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', d['verdict_check'].get('mismatches_vs_construction'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/trace_c4h -o c4h -- python3 $R/bench.py --workload c4h --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { echo "trace failed"; tail -n 20 $O/trace.log; exit 1; }
find /tmp/trace_c4h -name "*kernel_trace.csv" -exec cp {} $O/c4h_kernel_trace.csv \;
find /tmp/trace_c4h -name "*memory_copy_trace.csv" -exec cp {} $O/c4h_memory_copy_trace.csv \;
