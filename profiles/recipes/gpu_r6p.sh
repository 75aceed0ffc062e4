# r06: id-slice lookahead A/B on c4h --components --inflight 2 and c4h --inflight 2 (alternating, x2)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6p
mkdir -p $O
cd $R
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 10 --warmup 2 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
C="--workload c4h --components --inflight 2"
L="--workload c4h --inflight 2"
run c4 "--workload c4" || exit 1
for k in 1 2; do
  CORDAHIP_TX_SLICE_AHEAD=1 run c_a1_$k "$C" && CORDAHIP_TX_SLICE_AHEAD=2 run c_a2_$k "$C" && CORDAHIP_TX_SLICE_AHEAD=3 run c_a3_$k "$C" && \
  CORDAHIP_TX_SLICE_AHEAD=1 run l_a1_$k "$L" && CORDAHIP_TX_SLICE_AHEAD=2 run l_a2_$k "$L" || exit 1
done
