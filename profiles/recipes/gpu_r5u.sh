# r05: the whole GPU suite and smoke on the current tree
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5u
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
