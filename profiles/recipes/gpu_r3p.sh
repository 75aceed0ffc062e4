# c4h signature chunk A/B on the dedicated-queue streams
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3p
mkdir -p $O
cd $R
for ch in ${CHUNKS:-131072 262144 156224 131072 262144 156224}; do
  i=$((i+1))
  CORDAHIP_TX_SIG_CHUNK=$ch CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload c4h --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4h_${ch}_$i.json 2> $O/trace_c4h_${ch}_$i.err || { echo "bench $ch failed"; tail -n 5 $O/trace_c4h_${ch}_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c4h_${ch}_$i.json'));print('c4h chunk $ch', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', d['verdict_check'].get('mismatches_vs_construction'))"
done
