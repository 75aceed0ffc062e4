# Round-4 GPU call n: kernel/copy trace of c4h on the two-stream pipeline (queue ids)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
BENCH_ARGS=--no-clock TAG=r4n_c4h WL=c4h STEPS=2 bash tools/gpu_trace.sh > /dev/null || { echo "trace failed"; exit 1; }
head -3 gpurun_out/trace/r4n_c4h_gaps.txt
