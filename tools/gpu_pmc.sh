# rocprofv3 PMC passes (one counter group per pass, each under its own KILL timeout)
# over one bench step: WL (c2|c3|c4), LOG2 batch size, TAG names the output.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_${TAG:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --workload ${WL:-c2} --batch-log2 ${LOG2:-22} --c4-txs ${C4TXS:-262144} --steps 1 --warmup 0 --no-cpu-baseline --no-clock"
i=0
for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc_$i -o p -- $BENCH > $O/pass$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
  find /tmp/pmc_$i -name "*counter_collection.csv" -exec cp {} $O/pass$i.csv \;
done
python3 $R/tools/pmc_summary.py $O/pass*.csv > $O/summary.json && cat $O/summary.json
