# Round-4 GPU call f: traces of the current host pipelines (c4h, c2h) with the
# library's own phase trace (CORDAHIP_TRACE) beside them
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_f
mkdir -p $O
cd $R
BENCH_ARGS=--no-clock TAG=r4f_c4h WL=c4h STEPS=2 bash tools/gpu_trace.sh > $O/trace_c4h.txt || { echo "trace c4h failed"; tail -5 $O/trace_c4h.txt; exit 1; }
head -4 $O/trace_c4h.txt
BENCH_ARGS=--no-clock TAG=r4f_c2h WL=c2h STEPS=2 bash tools/gpu_trace.sh > $O/trace_c2h.txt || { echo "trace c2h failed"; tail -5 $O/trace_c2h.txt; exit 1; }
head -4 $O/trace_c2h.txt
CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload c2h --steps 2 --warmup 1 --no-cpu-baseline --no-clock > $O/c2h_hosttrace.json 2> $O/c2h_hosttrace.err || { echo "c2h host trace failed"; tail -5 $O/c2h_hosttrace.err; exit 1; }
grep cordahip $O/c2h_hosttrace.err | tail -12
