# C5 A/B over the stream pipeline's chunk size (CORDAHIP_STREAM_CHUNK, lanes
# per chunk, both sections together): one short C5 bench per value, on one box.
# Usage (GPU box): CHUNKS="2097152 4194304 8388608" bash tools/gpu_c5_chunk_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c5ab
mkdir -p $O
cd $R
for c in ${CHUNKS:-2097152 4194304 8388608 16777216}; do
  CORDAHIP_STREAM_CHUNK=$c timeout -k 10 300 python bench.py --workload c5 --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline \
    > $O/bench_c5_$c.json 2> $O/bench_c5_$c.err || { echo "bench chunk $c failed"; tail -20 $O/bench_c5_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c5_$c.json'));print('chunk', $c, round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],1), 'ms', d['verdict_check'])"
done
