# Round-4 GPU call d: FP64 field A/B microbenchmark; kernel/copy traces of the
# new host pipelines (c4h, c2h)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_d
mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/microbench/fp64_field_check.py 256 $O/r04_fp64_field_ab.json > $O/fp64.txt 2>&1 || { echo "fp64 A/B failed"; tail -20 $O/fp64.txt; exit 1; }
cat $O/fp64.txt
BENCH_ARGS=--no-clock TAG=r4d_c4h WL=c4h STEPS=2 bash tools/gpu_trace.sh > $O/trace_c4h.txt || { echo "trace c4h failed"; tail -5 $O/trace_c4h.txt; exit 1; }
head -12 $O/trace_c4h.txt
BENCH_ARGS=--no-clock TAG=r4d_c2h WL=c2h STEPS=2 bash tools/gpu_trace.sh > $O/trace_c2h.txt || { echo "trace c2h failed"; tail -5 $O/trace_c2h.txt; exit 1; }
head -8 $O/trace_c2h.txt
