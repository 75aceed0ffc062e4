# r05: kernel + copy trace of c4h (synthetic 838-B leaves, current defaults) for its PCIe busy time
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/t5o -o t -- python3 $R/bench.py --workload c4h --steps 1 --warmup 1 --no-cpu-baseline --no-clock > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
find /tmp/t5o -name "*kernel_trace.csv" -exec cp {} $O/c4h_kernel_trace.csv \;
find /tmp/t5o -name "*memory_copy_trace.csv" -exec cp {} $O/c4h_memory_copy_trace.csv \;
python3 $R/tools/c4h_timeline.py $O/c4h_kernel_trace.csv $O/c4h_memory_copy_trace.csv > $O/timeline.txt && head -8 $O/timeline.txt
