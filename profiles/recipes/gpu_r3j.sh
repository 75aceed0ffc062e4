# ECDSA formula A/B per kernel: for each tag in $TAGS swap ab_libs/<tag> in,
# run the ECDSA GPU tests, rocprofv3 kernel stats of a C3 bench (2^24 lanes)
# and an SQ_INSTS_VALU pass on a 2^22 C3 step
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3j
mkdir -p $O
cp $R/corda_amd/libcordahip.so $O/orig.so
cd /tmp && export TMPDIR=/tmp
for v in $TAGS; do
  cp $R/ab_libs/$v/libcordahip.so $R/corda_amd/libcordahip.so
  (cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_ecdsa.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1) || { echo "pytest $v failed"; tail -n 30 $O/pytest_$v.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$v -o p -- python3 $R/bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_$v.json 2> $O/prof_$v.err || { echo "prof $v failed"; tail -n 20 $O/prof_$v.err; exit 1; }
  find /tmp/prof_$v -name "*kernel_stats.csv" -exec cp {} $O/${v}_kernel_stats.csv \;
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d /tmp/pmc_$v -o p -- python3 $R/bench.py --workload c3 --batch-log2 22 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -n 5 $O/pmc_$v.log; exit 1; }
  find /tmp/pmc_$v -name "*counter_collection.csv" -exec cp {} $O/${v}_pmc.csv \;
  python3 - <<PY
import csv, json, collections
d = json.load(open("$O/bench_$v.json"))
r = list(csv.DictReader(open("$O/${v}_kernel_stats.csv")))
k = {x['Name'][:40]: round(float(x['AverageNs']) / 1e6, 3) for x in r if 'ecdsa' in x['Name']}
pm = collections.defaultdict(float)
for x in csv.DictReader(open("$O/${v}_pmc.csv")):
    if x.get('Counter_Name') == 'SQ_INSTS_VALU' and 'ladder' in x.get('Kernel_Name', ''):
        pm[x['Kernel_Name'][:40]] += float(x['Counter_Value'])
print("$v", round(d['value'] / 1e6, 2), "M/s", d['verdict_check']['mismatches_vs_construction'], d['verdict_check']['mismatches_vs_oracle_open_lanes'], k, dict(pm))
PY
done
cp $O/orig.so $R/corda_amd/libcordahip.so
