# One profiling pass over the current tree (run through gpurun): rocprofv3
# kernel-trace stats of the C2 and C3 bench, the PMC passes of
# tools/gpu_pmc.sh for both, and the VALU counter calibration on
# tools/microbench/valu_rates.hip (binary prebuilt at ab_libs/valu_rates).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for wl in ${KT_WLS:-c2 c3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$wl -o kt -- python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_$wl.json 2> $O/kt_$wl.err || { echo "kernel trace $wl failed"; tail -5 $O/kt_$wl.err; exit 1; }
  find /tmp/kt_$wl -name "*kernel_stats.csv" -exec cp {} $O/${wl}_kernel_stats.csv \;
  echo "kt $wl done"
done
for wl in ${PMC_WLS:-c3 c2}; do
  WL=$wl TAG=$wl bash $R/tools/gpu_pmc.sh > $O/pmc_$wl.log 2>&1 || { echo "pmc $wl failed"; tail -5 $O/pmc_$wl.log; exit 1; }
  echo "pmc $wl done"
done
if [ "${CAL:-1}" = 1 ] && [ -x $R/ab_libs/valu_rates ]; then
  timeout -k 10 120 $R/ab_libs/valu_rates > $O/valu_rates.jsonl || { echo "valu_rates failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/cal -o cal -- $R/ab_libs/valu_rates > $O/cal.log 2>&1 || { echo "calibration pmc failed"; tail -5 $O/cal.log; exit 1; }
  find /tmp/cal -name "*counter_collection.csv" -exec cp {} $O/cal.csv \;
  python3 $R/tools/pmc_summary.py --all $O/cal.csv > $O/cal_summary.json
  python3 $R/tools/pmc_calibrate.py $O/valu_rates.jsonl $O/cal_summary.json > $O/calibration.json
  echo "calibration done"
fi
