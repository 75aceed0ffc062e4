# r06: kryo_hash with shape-grouped blocks (256 items of one kind per block, lanes
# grouped by template in LDS, the scalar path for single-template waves) against the
# previous kernel (ab_libs/old): id-chain tests on the new library, then alternating
# rocprof'd c4 --device-encode runs and c4h --components --inflight 2 runs
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6v
mkdir -p $O
cd $R
cp corda_amd/libcordahip.so $O/new.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_txcomp.py tests/test_gpu_kryo_fuzz.py tests/test_gpu_kryo.py tests/test_gpu_memory.py -x -q --timeout 300 --timeout-method thread -k "not 2_29" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
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
print("$1", round(d["value"] / 1e6, 2), {k: round(v, 3) for k, v in r.items() if "kryo_hash" in k or "kryo_shape" in k},
      {k: v for k, v in d["verdict_check"].items() if "mismatch" in k and v})
PY
}
run() {
  timeout -k 10 400 python -u $R/bench.py --no-cpu-baseline --no-clock --steps 20 --warmup 4 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
use() { cp $1 $R/corda_amd/libcordahip.so; }
for rep in 1 2; do
  use $O/new.so && prof de_new_$rep "--workload c4 --device-encode" && use $R/ab_libs/old/libcordahip.so && prof de_old_$rep "--workload c4 --device-encode" || exit 1
done
for rep in 1 2; do
  use $O/new.so && run hc_new_$rep "--workload c4h --components --inflight 2" && use $R/ab_libs/old/libcordahip.so && run hc_old_$rep "--workload c4h --components --inflight 2" || exit 1
done
use $O/new.so
