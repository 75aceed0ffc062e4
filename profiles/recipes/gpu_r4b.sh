# Round-4 GPU call b: available PMC counters, kernel/copy traces of the boundary
# paths (c2h, c4h), C2 PMC passes on the round-4 library.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1 || echo "counter list failed (rc $?)"
cd $R
BENCH_ARGS=--no-clock TAG=r4_c2h WL=c2h STEPS=2 bash tools/gpu_trace.sh > $O/trace_c2h.txt || { echo "trace c2h failed"; tail -5 $O/trace_c2h.txt; exit 1; }
tail -25 $O/trace_c2h.txt
BENCH_ARGS=--no-clock TAG=r4_c4h WL=c4h STEPS=2 bash tools/gpu_trace.sh > $O/trace_c4h.txt || { echo "trace c4h failed"; tail -5 $O/trace_c4h.txt; exit 1; }
tail -25 $O/trace_c4h.txt
TAG=r4_c2 WL=c2 LOG2=22 bash tools/gpu_pmc.sh > $O/pmc_c2.txt || { echo "pmc c2 failed"; tail -5 $O/pmc_c2.txt; exit 1; }
cp -r $R/gpurun_out/pmc_r4_c2 $O/
tail -30 $O/pmc_c2.txt
