# r06: c3h with the generic batches' ECDSA chunk alternation on / off
# (CORDAHIP_EC_ALTERNATE), one and two calls in flight, alternating on one box;
# two warmup steps, so both transaction sets have grown their stages before timing
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6am}
mkdir -p $O
cd $R
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 6 --warmup 2 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
for rep in 1 2; do
  run c3_$rep "--workload c3" && run h1_on_$rep "--workload c3h" && CORDAHIP_EC_ALTERNATE=0 run h1_off_$rep "--workload c3h" && \
  run h2_on_$rep "--workload c3h --inflight 2" && CORDAHIP_EC_ALTERNATE=0 run h2_off_$rep "--workload c3h --inflight 2" || exit 1
done
