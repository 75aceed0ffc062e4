# r06 final evidence pass, part 2: every other workload's bench line once (the
# signed-tx boundary lines at two calls in flight with 40 steps, so the line is the
# steady state rather than the first calls' table builds and buffer growth).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6final
mkdir -p $O
cd $R
line() {
  t=$1; shift
  timeout -k 10 600 python -u bench.py "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));print('$t', round(d['value']/1e6,2), round(d['ms_per_step'],2), d.get('clock_ghz') and round(d['clock_ghz'],3), d.get('valu_busy') and round(d['valu_busy']['valu_busy'],3), d.get('device_mem_gb'), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k})"
}
line c4 --workload c4 && line c4h2 --workload c4h --inflight 2 --steps 40 --warmup 6 && \
line c4hc2 --workload c4h --components --inflight 2 --steps 40 --warmup 6 && line c4de --workload c4 --device-encode && \
line c1 --workload c1 && line c3 --workload c3 && line c5 --workload c5 && line c2h --workload c2h && \
line c3h --workload c3h && line c4h --workload c4h && line c4hc --workload c4h --components && \
line c2h2 --workload c2h --inflight 2 --steps 8 --warmup 2 && line c3h2 --workload c3h --inflight 2 --steps 8 --warmup 2
