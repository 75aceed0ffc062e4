# r05: fabric bytes of the component-level id chain (kryo_shape, kryo_hash, merkle_root) inside
# c4h --components calls: FETCH_SIZE and WRITE_SIZE passes, per transaction from each
# dispatch's grid (one thread per component, 5 per transaction)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ai
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --workload c4h --components --steps 1 --warmup 1 --no-cpu-baseline --no-clock"
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc5ai_$i -o p -- $B > $O/pass$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
  find /tmp/pmc5ai_$i -name "*counter_collection.csv" -exec cp {} $O/pass$i.csv \;
done
python3 - <<PY
import csv, collections, json
out = {}
for i, c in ((1, "FETCH_SIZE"), (2, "WRITE_SIZE")):
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for r in csv.DictReader(open("$O/pass%d.csv" % i)):
        n = r["Kernel_Name"]
        k = next((x for x in ("kryo_shape", "kryo_hash", "merkle_root", "ed25519_prep", "ed25519_ladder") if x in n), None)
        if not k or r["Counter_Name"] != c:
            continue
        g = float(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
        agg[k][0] += float(r["Counter_Value"]) * 1024 * (2 if c == "FETCH_SIZE" else 1)
        agg[k][1] += g
        agg[k][2] += 1
    for k, (b, g, d) in agg.items():
        per = b / g * (5 if k.startswith("kryo") else 1) if g else None  # kryo: per tx (5 items); others: per thread
        out.setdefault(k, {})[c.lower() + "_bytes_per_unit"] = per
        out[k]["dispatches"] = d
print(json.dumps(out, indent=1))
json.dump(out, open("$O/r05_pmc_txcomp_chain.json", "w"), indent=1)
PY
