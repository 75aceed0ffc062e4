# r06: host signed-tx pipeline knobs at --inflight 2 (signature chunk 98,304 vs 2^17,
# two id slices ahead), alternating on one box, steps 20 / warmup 4
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6x
mkdir -p $O
cd $R
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 20 --warmup 4 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
HC="--workload c4h --components --inflight 2"
H="--workload c4h --inflight 2"
for rep in 1 2; do
  run c4_$rep "--workload c4" && run hc_base_$rep "$HC" && CORDAHIP_TX_SIG_CHUNK=98304 run hc_c98_$rep "$HC" && \
  CORDAHIP_TX_SLICE_AHEAD=2 run hc_a2_$rep "$HC" && CORDAHIP_TX_SIG_CHUNK=98304 CORDAHIP_TX_SLICE_AHEAD=2 run hc_c98a2_$rep "$HC" && \
  run h_base_$rep "$H" && CORDAHIP_TX_SIG_CHUNK=98304 run h_c98_$rep "$H" && CORDAHIP_TX_SLICE_AHEAD=2 run h_a2_$rep "$H" || exit 1
done
