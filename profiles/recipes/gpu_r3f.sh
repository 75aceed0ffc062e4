# c2h (2^22 chunks), c4h at 2 and 4 tx slices, then a slice of the agreement sweep
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r3f}
mkdir -p $O
cd $R
run() {  # name, env..., workload
  local name=$1; shift
  env "$@" CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$name.json 2> $O/trace_$name.err || { echo "bench $name failed"; tail -5 $O/trace_$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$name.json'));print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', d['verdict_check'].get('mismatches_vs_construction'), d['verdict_check'].get('mismatches_vs_oracle_open_lanes'))"
  grep "signed tx\|shard done" $O/trace_$name.err | tail -3
}
WL=c2h run c2h CORDAHIP_X=1 && WL=c4h run c4h_s2 CORDAHIP_TX_SLICES=2 && WL=c4h run c4h_s4 CORDAHIP_TX_SLICES=4 && WL=c4h run c4h_s1 CORDAHIP_TX_SLICES=1 || exit 1
if [ -n "$ED$EC" ]; then
  timeout -k 10 ${SWEEP_S:-900} python -u tools/agree_1e9.py --oracle-all --ed ${ED:-0} --ec ${EC:-0} --first ${FIRST:-0} --threads 16 --log $O/agree_log.jsonl > $O/agree.out 2>&1; rc=$?
  tail -3 $O/agree.out
  exit $rc
fi
