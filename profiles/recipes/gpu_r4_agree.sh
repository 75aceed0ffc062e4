# Round-4 agreement sweep slice on the GPU box: every lane oracle-checked
# (tools/agree_1e9.py --oracle-all). SLICE names the log; ARGS selects batches,
# e.g. ARGS="--ed 0 --ec 1 --stream 4 --first 4". RERUN_ED=k first re-runs
# dense Ed25519 batches 0..k-1 (counted in r03) into a separate log.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/agree_r04
mkdir -p $O
cd $R
if [ -n "$SANITY" ]; then
  timeout -k 10 300 python -u tools/agree_1e9.py --log2 16 --ed 0 --ec 0 --stream 1 --first 900 --oracle-all > $O/sanity.log 2>&1 || { echo "sanity failed"; tail -20 $O/sanity.log; exit 1; }
  tail -1 $O/sanity.log
fi
if [ -n "$RERUN_ED" ]; then
  timeout -k 10 600 python -u tools/agree_1e9.py --ed $RERUN_ED --ec 0 --stream 0 --first 0 --oracle-all --log $O/rerun_ed_r03_0-$((RERUN_ED-1)).jsonl > $O/rerun.log 2>&1 || { echo "rerun failed"; tail -20 $O/rerun.log; exit 1; }
  tail -1 $O/rerun.log
fi
timeout -k 10 ${LIMIT:-1000} python -u tools/agree_1e9.py $ARGS --oracle-all --log $O/$SLICE.jsonl > $O/$SLICE.log 2>&1 || { echo "slice failed"; tail -20 $O/$SLICE.log; exit 1; }
tail -1 $O/$SLICE.log
