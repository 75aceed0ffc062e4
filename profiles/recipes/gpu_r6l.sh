# r06: per-device NUMA pools A/B (CORDAHIP_NUMA=0 vs bound) on c2h and c4h --inflight 2, with c4 as the box
# reference; pack_bench with one bound pool per simulated device
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6l
mkdir -p $O
cd $R
g++ -O2 -std=c++17 -pthread -o /tmp/pack_bench tools/pack_bench.cpp || exit 1
for p in 1 2 8; do timeout -k 10 120 /tmp/pack_bench $((1<<22)) 16 $p | tee -a $O/pack_pools.jsonl || exit 1; done
timeout -k 10 120 /tmp/pack_bench $((1<<22)) 16 | tee $O/pack_threads.jsonl || exit 1
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 8 --warmup 2 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k})"
}
run c4 "--workload c4" || exit 1
for k in 1 2; do
  CORDAHIP_NUMA=0 run c4h2_unbound$k "--workload c4h --inflight 2" && run c4h2_bound$k "--workload c4h --inflight 2" && \
  CORDAHIP_NUMA=0 run c2h_unbound$k "--workload c2h" && run c2h_bound$k "--workload c2h" || exit 1
done
