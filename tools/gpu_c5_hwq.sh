set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5q
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5q/b_$q.json 2> gpurun_out/c5q/b_$q.err || { echo "bench q=$q failed"; tail -5 gpurun_out/c5q/b_$q.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c5q/b_$q.json'));print('hwq', $q, round(d['value']/1e6,2), round(d['ms_per_step'],1), d['verdict_check'])"
done
