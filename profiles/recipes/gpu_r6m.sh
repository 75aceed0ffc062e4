# r06: memory budget / idle release tests, then the tx, runtime and host-batch tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6m
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_memory.py tests/test_gpu_csr.py tests/test_gpu_runtime.py tests/test_gpu_tx.py tests/test_gpu_host_batch.py tests/test_gpu_stream.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED" $O/pytest.log | grep -c PASSED; tail -1 $O/pytest.log
