# r06: the id / encoder kernels' stream on N spread CUs (CORDAHIP_ID_CUS), the
# verification streams on all: c4h --components and c4h at --inflight 2, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ae
mkdir -p $O
cd $R
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 20 --warmup 4 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
HC="--workload c4h --components --inflight 2"
H="--workload c4h --inflight 2"
for rep in 1 2; do
  run hc_all_$rep "$HC" && CORDAHIP_ID_CUS=128 run hc_128_$rep "$HC" && CORDAHIP_ID_CUS=64 run hc_64_$rep "$HC" && \
  CORDAHIP_ID_CUS=32 run hc_32_$rep "$HC" && run h_all_$rep "$H" && CORDAHIP_ID_CUS=64 run h_64_$rep "$H" || exit 1
done
