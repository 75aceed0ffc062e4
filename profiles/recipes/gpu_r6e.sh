# r06: kryo_hash A/B (occupancy variants, CORDAHIP_KRYO_HASH_WAVES) on c4 --device-encode, kernel summaries
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in 4 5 6 4b; do
  export CORDAHIP_KRYO_HASH_WAVES=${w%b}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_$w -o w$w -- python3 $R/bench.py --no-cpu-baseline --no-clock --steps 6 --warmup 2 --workload c4 --device-encode > $O/prof_$w.log 2>&1 || { echo "prof $w failed"; tail -20 $O/prof_$w.log; exit 1; }
  find /tmp/p_$w -name "*kernel_stats.csv" -exec cp {} $O/w${w}_kernel_stats.csv \;
  python3 - <<PY
import csv, json
r = {x["Name"].split("(")[0][-24:]: x for x in csv.DictReader(open("$O/w${w}_kernel_stats.csv"))}
line = [l for l in open("$O/prof_$w.log") if l.startswith("{")]
d = json.loads(line[-1]) if line else {}
print("waves $w", {k: round(float(v["AverageNs"]) / 1e6, 3) for k, v in r.items() if "kryo" in k or "merkle" in k}, round(d.get("value", 0) / 1e6, 2), d.get("verdict_check", {}).get("mismatches_vs_leaf_path"))
PY
done
