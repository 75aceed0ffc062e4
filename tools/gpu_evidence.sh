# Bench line + rocprofv3 kernel stats of each workload in WLS on ONE box, so the
# bench's event-timed kernel_ms and the rocprof averages come from the same
# hardware (boxes differ by up to ~7% in sustained clock).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/evidence
mkdir -p $O
cd $R
for wl in ${WLS:-c2 c3 c5}; do
  timeout -k 10 600 python -u bench.py --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo "bench $wl failed"; tail -20 $O/bench_$wl.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$wl.json'));print('$wl', round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],2), 'ms', d['verdict_check'])"
  TAG=ev_$wl WL=$wl bash tools/gpu_prof.sh > $O/prof_$wl.txt || { echo "prof $wl failed"; exit 1; }
  cp gpurun_out/prof/ev_${wl}_kernel_stats.csv $O/
  head -4 $O/prof_$wl.txt
done
