# Round-4 GPU call k: c4h host-phase trace and kernel/copy trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_k
mkdir -p $O
cd $R
CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload c4h --steps 2 --warmup 1 --no-cpu-baseline --no-clock > $O/c4h.json 2> $O/c4h.err || { echo "c4h failed"; tail -5 $O/c4h.err; exit 1; }
grep cordahip $O/c4h.err | tail -23
BENCH_ARGS=--no-clock TAG=r4k_c4h WL=c4h STEPS=2 bash tools/gpu_trace.sh > $O/trace_c4h.txt || { echo "trace c4h failed"; tail -5 $O/trace_c4h.txt; exit 1; }
head -3 $O/trace_c4h.txt
