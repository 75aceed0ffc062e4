# r06 final evidence pass (one per round), part 1: the whole GPU suite and smoke,
# the driver's default bench line (C2) and its rocprofv3 kernel summary.
# Part 2 (tools/gpu_final_r6b.sh): every other workload's line once.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6final
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|passed|failed" $O/pytest_gpu.log | tail -20; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 failed"; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', round(d['value']/1e6,2), round(d['ms_per_step'],2), d['clock']['clock_ghz'], round(d['roofline']['frac'],3), d['verdict_check'])"
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pfinal
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pfinal -o c2 -- python3 $R/bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || { echo "prof failed"; tail -20 $O/prof_c2.log; exit 1; }
find /tmp/pfinal -name "*kernel_stats.csv" -exec cp {} $O/r06_c2_kernel_stats.csv \;
grep -h '^{' $O/prof_c2.log > $O/prof_c2_bench_line.json || true
python3 - <<PY
import csv, json
r = list(csv.DictReader(open("$O/r06_c2_kernel_stats.csv")))
for x in sorted(r, key=lambda x: -float(x["TotalDurationNs"]))[:4]:
    print(x["Name"][:60], x["Calls"], round(float(x["AverageNs"]) / 1e6, 3))
d = json.loads(open("$O/prof_c2_bench_line.json").read().splitlines()[-1])
print("kernel_ms in the profiled run's own line", round(d["roofline"]["kernel_ms"], 2))
PY
