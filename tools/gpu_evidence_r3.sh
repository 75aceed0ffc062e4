# Round-3 evidence from ONE box: bench lines (roofline + cpu_baseline) of every
# workload, rocprofv3 kernel stats of the device workloads, and the C5 PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ev3
mkdir -p $O
cd $R
for wl in ${WLS:-c2 c3 c4 c5 c1 c2h c3h c4h}; do
  timeout -k 10 420 python -u bench.py --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo "bench $wl failed"; tail -20 $O/bench_$wl.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$wl.json'));c=d['verdict_check'];print('$wl', round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],2), 'ms frac', round(d['roofline']['frac'],3), 'traffic', d['roofline']['traffic'] is not None, 'mism', c.get('mismatches_vs_construction'), c.get('mismatches_vs_oracle_open_lanes'), 'cpu', round(d.get('cpu_baseline',{}).get('value',0)))"
done
for wl in ${PROF:-c2 c3 c4 c5}; do
  TAG=ev3_$wl WL=$wl bash tools/gpu_prof.sh > $O/prof_$wl.txt || { echo "prof $wl failed"; tail -5 $O/prof_$wl.txt; exit 1; }
  cp gpurun_out/prof/ev3_${wl}_kernel_stats.csv $O/
  head -6 $O/prof_$wl.txt
done
if [ -n "$PMC" ]; then
  TAG=c5 WL=c5 LOG2=22 bash tools/gpu_pmc.sh > $O/pmc_c5.txt || { echo "pmc failed"; tail -5 $O/pmc_c5.txt; exit 1; }
  cp -r gpurun_out/pmc_c5 $O/
fi
