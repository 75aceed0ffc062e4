# r05 final evidence pass (one per round): the GPU suite and smoke, the driver's default bench
# line (C2) with its rocprofv3 kernel summary, and every other workload's line once.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5final
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 failed"; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', round(d['value']/1e6,2), d['ms_per_step'], d['clock']['clock_ghz'], d['roofline']['frac'])"
for wl in "c1" "c3" "c4" "c5" "c2h" "c3h" "c4h" "c4h --components" "c4 --device-encode"; do
  t=$(echo $wl | tr -d ' -')
  timeout -k 10 600 python -u bench.py --workload $wl > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $wl failed"; tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));print('$t', round(d['value']/1e6,2), d['clock']['clock_ghz'], {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k})"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pfinal -o c2 -- python3 $R/bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || { echo "prof failed"; tail -20 $O/prof_c2.log; exit 1; }
find /tmp/pfinal -name "*kernel_stats.csv" -exec cp {} $O/r05_c2_kernel_stats.csv \;
grep -h '^{' $O/prof_c2.log > $O/prof_c2_bench_line.json || true
python3 - <<PY
import csv
r = list(csv.DictReader(open("$O/r05_c2_kernel_stats.csv")))
for x in sorted(r, key=lambda x: -float(x["TotalDurationNs"]))[:4]:
    print(x["Name"][:60], x["Calls"], round(float(x["AverageNs"]) / 1e6, 3))
PY
