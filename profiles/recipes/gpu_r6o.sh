# r06: c4h --components --inflight 2 knobs A/B (one box, alternating), c4 as the reference
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6o
mkdir -p $O
cd $R
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 10 --warmup 2 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
C="--workload c4h --components --inflight 2"
run c4 "--workload c4" && run base1 "$C" && \
CORDAHIP_TX_SPLIT_PREP=1 run split1 "$C" && CORDAHIP_TX_SLICE_AHEAD=2 run ahead2 "$C" && \
CORDAHIP_TX_SIG_CHUNK=65536 run chunk16 "$C" && CORDAHIP_KRYO_HASH_WAVES=4 run waves4 "$C" && \
run base2 "$C" && CORDAHIP_TX_SPLIT_PREP=1 run split2 "$C" && run inflight3 "--workload c4h --components --inflight 3"
