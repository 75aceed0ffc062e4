# r06: device signed-tx paths with the ids first and the fused Ed25519 prep (no split
# launches when nothing runs beside them): the device-path tests, then c4 and
# c4 --device-encode with rocprofv3 kernel stats, twice each
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6s
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_txcomp.py tests/test_gpu_runtime.py -x -q --timeout 300 --timeout-method thread -k "not 2_29" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
prof() {
  rm -rf /tmp/p_$1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_$1 -o p -- python3 $R/bench.py $2 --no-cpu-baseline --no-clock --steps 10 --warmup 2 > $O/b_$1.json 2> $O/b_$1.err || { echo "prof $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  find /tmp/p_$1 -name "*kernel_stats.csv" -exec cp {} $O/$1_kernel_stats.csv \;
  python3 - <<PY
import csv, json
d = json.loads([l for l in open("$O/b_$1.json") if l.startswith("{")][-1])
r = {x["Name"].replace("(anonymous namespace)::", "").split("(")[0][-30:]: float(x["AverageNs"]) / 1e6 for x in csv.DictReader(open("$O/$1_kernel_stats.csv"))}
print("$1", round(d["value"] / 1e6, 2), {k: round(v, 3) for k, v in r.items() if "prep" in k or "ladder" in k or "kryo_hash" in k},
      {k: v for k, v in d["verdict_check"].items() if "mismatch" in k and v})
PY
}
prof c4 "--workload c4" && prof c4de "--workload c4 --device-encode" && prof c4b "--workload c4" && prof c4deb "--workload c4 --device-encode"
