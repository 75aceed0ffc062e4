# Round-4 GPU call t: the GPU Kryo encoder -- its parity tests, then C4 with the
# leaves encoded on the GPU every step beside C4 with host-made native leaves and
# plain C4, then rocprof kernel stats of the device-encode step
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_${TAG:-t}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kryo.py tests/test_gpu_tx.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
run() {  # name, workload args
  timeout -k 10 400 python -u bench.py $2 --steps 5 --warmup 1 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -8 $O/$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$1.json'));c=d['verdict_check'];print('$1', round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],2), 'ms clk', round(d.get('clock_ghz') or 0,3), c)"
}
run c4_devenc "--workload c4 --device-encode" || exit 1
[ -z "$SKIP_REF" ] && { run c4_native "--workload c4 --native-leaves" || exit 1; }
[ -z "$SKIP_REF" ] && { run c4 "--workload c4" || exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_devenc -o devenc -- python3 $R/bench.py --workload c4 --device-encode --steps 2 --warmup 1 --no-cpu-baseline --no-clock > $O/prof_devenc.log 2>&1 || { echo "prof failed"; tail -5 $O/prof_devenc.log; exit 1; }
find /tmp/prof_devenc -name "*kernel_stats.csv" -exec cp {} $O/devenc_kernel_stats.csv \;
python3 - <<PY
import csv
r=list(csv.DictReader(open("$O/devenc_kernel_stats.csv")))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:10]: print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e6,3))
PY
