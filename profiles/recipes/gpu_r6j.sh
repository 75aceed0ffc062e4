# r06: the whole GPU suite on the ABI-4 library
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6j
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread 2>&1 | tee $O/pytest_gpu.log | grep -E "PASSED|FAILED|ERROR|passed|failed" | tail -100
