# rocprofv3 kernel stats of one bench workload for each library variant in $TAGS
# (ab_libs/<tag>/libcordahip.so from tools/build_ab.sh): per-kernel time split.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/profab
mkdir -p $O
cp $R/corda_amd/libcordahip.so $O/orig.so
cd /tmp && export TMPDIR=/tmp
for v in $TAGS; do
  cp $R/ab_libs/$v/libcordahip.so $R/corda_amd/libcordahip.so
  P=/tmp/profab_$v
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o $v -- python3 $R/bench.py --workload ${WL:-c2} --steps 2 --warmup 1 --no-cpu-baseline > $O/$v.log 2>&1 || { echo "prof $v failed"; tail -20 $O/$v.log; exit 1; }
  find $P -name "*kernel_stats.csv" -exec cp {} $O/${v}_kernel_stats.csv \;
  python3 - <<PY
import csv
r=list(csv.DictReader(open("$O/${v}_kernel_stats.csv")))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:5]: print("$v", x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e6,3))
PY
done
cp $O/orig.so $R/corda_amd/libcordahip.so
