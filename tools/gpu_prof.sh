# rocprofv3 kernel stats of one bench workload: WL (c2|c3|c4), TAG names the output
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof
P=/tmp/prof_$TAG
mkdir -p $O $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o $TAG -- python3 $R/bench.py --workload ${WL:-c2} --steps 2 --warmup 1 --no-cpu-baseline --no-clock > $O/$TAG.log 2>&1 || { echo "prof failed"; tail -20 $O/$TAG.log; exit 1; }
find $P -name "*kernel_stats.csv" -exec cp {} $O/${TAG}_kernel_stats.csv \;
python3 - <<PY
import csv
r=list(csv.DictReader(open("$O/${TAG}_kernel_stats.csv")))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:8]: print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e6,3), x['Percentage'])
PY
