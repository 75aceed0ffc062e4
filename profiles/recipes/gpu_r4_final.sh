# Round-4 end rehearsal on the committed tree: the whole GPU test suite, smoke(),
# and the default bench line exactly as the driver runs them.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_final7
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -n 40 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -8 $O/bench.err; exit 1; }
cat $O/bench.json
