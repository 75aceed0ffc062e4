# r05: request-size split of the Kryo encoder's L2-fabric traffic (calibrates FETCH_SIZE x2
# for its access widths): TCC_EA0_RDREQ by size, WRREQ by size, L2 hits / misses
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kryo_dev_bench.py --txs 262144 --calls 2"
i=0
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc5m_$i -o p -- $K > $O/pass$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
  find /tmp/pmc5m_$i -name "*counter_collection.csv" -exec cp {} $O/pass$i.csv \;
done
python3 - <<PY
import csv, collections
d = collections.defaultdict(lambda: collections.defaultdict(float))
last = {}
for i in (1, 2, 3):
    rows = list(csv.DictReader(open("$O/pass%d.csv" % i)))
    for r in rows:
        n = r["Kernel_Name"]
        if "kryo_" not in n: continue
        k = n.split("kryo_")[1].split("_kernel")[0]
        did = int(r["Dispatch_Id"])
        key = (i, k)
        if key not in last or did > last[key]: last[key] = did
    for r in rows:
        n = r["Kernel_Name"]
        if "kryo_" not in n: continue
        k = n.split("kryo_")[1].split("_kernel")[0]
        if int(r["Dispatch_Id"]) == last[(i, k)]:
            d[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in d.items():
    print(k, {a: round(b / 262144, 2) for a, b in v.items()})
PY
