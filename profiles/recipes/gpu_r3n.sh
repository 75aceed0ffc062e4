# stream/queue placement A/B (CORDAHIP_IDCOPY modes: 1 id-copy stream created
# last, 3 created first, 4 CU-masked dedicated queues + high-priority ECDSA
# stream, 5 all CU-masked) on c4h, c5, c2h; then a kernel trace of c5 in mode 4
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3n
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_stream.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest.log; exit 1; }
CORDAHIP_IDCOPY=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_stream.py tests/test_gpu_host_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest4.log 2>&1 || { echo "pytest mode 4 failed"; tail -n 30 $O/pytest4.log; exit 1; }
tail -n 1 $O/pytest4.log
for v in ${MODES:-4 5 3 1}; do
  for wl in c4h c5 c2h; do
    CORDAHIP_IDCOPY=$v timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_${wl}_$v.json 2> $O/err_${wl}_$v.err || { echo "bench $wl $v failed"; tail -n 5 $O/err_${wl}_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${wl}_$v.json'));print('$wl mode $v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', d['verdict_check'].get('mismatches_vs_construction'))"
  done
done
cd /tmp && export TMPDIR=/tmp
CORDAHIP_IDCOPY=4 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr4 -o c5 -- python3 $R/bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/trace.log 2>&1 || { echo "trace failed"; tail -n 20 $O/trace.log; exit 1; }
find /tmp/tr4 -name "*kernel_trace.csv" -exec cp {} $O/c5_mode4_kernel_trace.csv \;
