# H2D bandwidth probe, then a slice of the fully oracle-checked agreement sweep
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r3g}
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 120 python -u tools/pcie_probe.py > $O/pcie.json 2> $O/pcie.err || { echo "probe failed"; tail -5 $O/pcie.err; exit 1; }
cat $O/pcie.json
timeout -k 10 ${SWEEP_S:-900} python -u tools/agree_1e9.py --oracle-all --ed ${ED:-0} --ec ${EC:-0} --first ${FIRST:-0} --threads 16 --log $O/agree_log.jsonl > $O/agree.out 2>&1; rc=$?
tail -3 $O/agree.out
exit $rc
