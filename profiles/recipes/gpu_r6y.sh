# r06: uniform id slices per call (CORDAHIP_TX_SLICES) for the host signed-tx
# paths at --inflight 2: fewer, larger id launches (the id waves hold VGPRs beside
# the ladders 84% of a c4h --components call at one slice per chunk)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6y
mkdir -p $O
cd $R
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 20 --warmup 4 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
HC="--workload c4h --components --inflight 2"
H="--workload c4h --inflight 2"
for rep in 1 2; do
  run hc_base_$rep "$HC" && CORDAHIP_TX_SLICES=2 run hc_s2_$rep "$HC" && CORDAHIP_TX_SLICES=4 run hc_s4_$rep "$HC" && \
  CORDAHIP_TX_SLICES=8 run hc_s8_$rep "$HC" && run h_base_$rep "$H" && CORDAHIP_TX_SLICES=4 run h_s4_$rep "$H" || exit 1
done
