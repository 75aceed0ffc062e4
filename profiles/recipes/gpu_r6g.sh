# r06: kryo_hash vs sha256_leaves at two batch sizes (kernel traces)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export CORDAHIP_KRYO_HASH_WAVES=5
for cfg in "c4 262144" "c4de 262144" "c4 1250000" "c4de 1250000"; do
  set -- $cfg
  a="--workload c4"; [ $1 = c4de ] && a="--workload c4 --device-encode"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_$1_$2 -o k -- python3 $R/bench.py --no-cpu-baseline --no-clock --steps 4 --warmup 1 --c4-txs $2 $a > $O/prof_$1_$2.log 2>&1 || { echo "prof $cfg failed"; tail -20 $O/prof_$1_$2.log; exit 1; }
  f=$(find /tmp/p_$1_$2 -name "*kernel_stats.csv")
  cp $f $O/$1_$2_kernel_stats.csv
  python3 - <<PY
import csv
for x in csv.DictReader(open("$f")):
    n = x["Name"]
    if any(k in n for k in ("kryo_hash", "kryo_shape", "sha256_leaves", "merkle_root", "ladder", "prep_half")):
        print("$cfg", n.replace("cordahip::(anonymous namespace)::", "")[:34], x["Calls"], round(float(x["AverageNs"]) / 1e6, 3))
PY
done
