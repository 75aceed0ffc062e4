# r05: signature chunk x slice lookahead sweep for c4h --components and c4h (id priority on)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5k
mkdir -p $O
cd $R
B="timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-clock"
run() {  # tag, workload args, env...
  local t=$1 w=$2; shift 2
  env "$@" $B $w > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -20 $O/$t.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$t.json')); v=d['verdict_check']; print('$t', round(d['value']/1e6,2), v.get('mismatches_vs_construction'), v.get('txid_mismatches_vs_device_path'))"
}
C="--workload c4h --components"
run comp_c17_a1 "$C" CORDAHIP_TX_SIG_CHUNK=131072 && run comp_c17_a2 "$C" CORDAHIP_TX_SIG_CHUNK=131072 CORDAHIP_TX_SLICE_AHEAD=2 && \
run comp_c18_a1 "$C" CORDAHIP_TX_SIG_CHUNK=262144 && run comp_c16_a2 "$C" CORDAHIP_TX_SLICE_AHEAD=2 && \
run comp_c17_a0 "$C" CORDAHIP_TX_SIG_CHUNK=131072 CORDAHIP_TX_SLICE_AHEAD=0 && run comp_c17_a1_again "$C" CORDAHIP_TX_SIG_CHUNK=131072 && \
run c4h_c16_a1 "--workload c4h" X=1 && run c4h_c17_a1 "--workload c4h" CORDAHIP_TX_SIG_CHUNK=131072 && run c4h_c16_a2 "--workload c4h" CORDAHIP_TX_SLICE_AHEAD=2 && \
run c4_again "--workload c4" X=1 && run c4de "--workload c4 --device-encode" X=1
