# c4h host trace + rocprof kernel/copy trace on the current library
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3o
mkdir -p $O
cd $R
CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload c4h --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4h.json 2> $O/trace_c4h.err || { echo "bench failed"; tail -n 5 $O/trace_c4h.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c4h.json'));print('c4h', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms')"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/tr -o c4h -- python3 $R/bench.py --workload c4h --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { echo "trace failed"; tail -n 20 $O/trace.log; exit 1; }
find /tmp/tr -name "*kernel_trace.csv" -exec cp {} $O/c4h_kernel_trace.csv \;
find /tmp/tr -name "*memory_copy_trace.csv" -exec cp {} $O/c4h_memory_copy_trace.csv \;
