# Final-kernel GPU suite + PMC passes for C3 (new ECDSA formulas) and C5
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3r
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -n 10 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
TAG=c3 WL=c3 LOG2=22 bash tools/gpu_pmc.sh > $O/pmc_c3.txt || { echo "pmc c3 failed"; tail -n 5 $O/pmc_c3.txt; exit 1; }
TAG=c5 WL=c5 LOG2=22 bash tools/gpu_pmc.sh > $O/pmc_c5.txt || { echo "pmc c5 failed"; tail -n 5 $O/pmc_c5.txt; exit 1; }
ls $R/gpurun_out/pmc_c3 $R/gpurun_out/pmc_c5
