# One GPU call: the full -m gpu suite on the tree's libcordahip.so, then the
# A/B of library variants in $TAGS (tools/gpu_ab.sh). Stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
[ -z "$TAGS" ] || bash tools/gpu_ab.sh
