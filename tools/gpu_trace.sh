# rocprofv3 kernel + memory-copy trace of one bench workload (no counters),
# then the busy/idle accounting of tools/trace_gaps.py over the timed steps.
# WL (default c5), TAG names the output; extra bench flags in BENCH_ARGS.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace
P=/tmp/trace_$TAG
mkdir -p $O $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $P -o $TAG -- python3 $R/bench.py --workload ${WL:-c5} --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline $BENCH_ARGS > $O/$TAG.log 2>&1 || { echo "trace failed"; tail -20 $O/$TAG.log; exit 1; }
K=$(find $P -name "*kernel_trace.csv" | head -1)
M=$(find $P -name "*memory_copy_trace.csv" | head -1)
cp $K $O/${TAG}_kernel_trace.csv
[ -n "$M" ] && cp $M $O/${TAG}_memory_copy_trace.csv
python3 $R/tools/trace_gaps.py $K $M --skip-before ${SKIP:-sign_kernel} | tee $O/${TAG}_gaps.txt
