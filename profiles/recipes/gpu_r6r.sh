# r06: kryo_hash wave-uniform scalar path: GPU tests of the id chains, then A/B on
# c4 --device-encode (rocprofv3 kernel stats, CORDAHIP_KRYO_HASH_UNIFORM=1/0, one box)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6r
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_txcomp.py tests/test_gpu_kryo_fuzz.py tests/test_gpu_memory.py tests/test_gpu_kryo.py -x -q --timeout 300 --timeout-method thread -k "not 2_29" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
prof() {
  rm -rf /tmp/p_$1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_$1 -o p -- python3 $R/bench.py --workload c4 --device-encode --no-cpu-baseline --no-clock --steps 10 --warmup 2 > $O/b_$1.json 2> $O/b_$1.err || { echo "prof $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  find /tmp/p_$1 -name "*kernel_stats.csv" -exec cp {} $O/$1_kernel_stats.csv \;
  python3 - <<PY
import csv, json
d = json.loads([l for l in open("$O/b_$1.json") if l.startswith("{")][-1])
r = {x["Name"].split("(")[0][-40:]: float(x["AverageNs"]) / 1e6 for x in csv.DictReader(open("$O/$1_kernel_stats.csv"))}
print("$1", round(d["value"] / 1e6, 2), {k: round(v, 3) for k, v in r.items() if "kryo_hash" in k or "shape" in k or "merkle" in k},
      {k: v for k, v in d["verdict_check"].items() if "mismatch" in k and v})
PY
}
CORDAHIP_KRYO_HASH_UNIFORM=1 prof u1 && CORDAHIP_KRYO_HASH_UNIFORM=0 prof u0 && CORDAHIP_KRYO_HASH_UNIFORM=1 prof u1b && \
CORDAHIP_KRYO_HASH_UNIFORM=1 CORDAHIP_KRYO_HASH_WAVES=4 prof u1w4 && CORDAHIP_KRYO_HASH_UNIFORM=0 prof u0b
