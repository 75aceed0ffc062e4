# r06: kernel summaries of c4 / c4h --inflight 2 / c4h --components --inflight 2 (rocprofv3 --stats)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
prof() {  # name, args
  timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/p_$1 -o $1 -- python3 $R/bench.py --no-cpu-baseline --no-clock --steps 6 --warmup 2 $2 > $O/prof_$1.log 2>&1 || { echo "prof $1 failed"; tail -20 $O/prof_$1.log; exit 1; }
  find /tmp/p_$1 -name "*kernel_stats.csv" -exec cp {} $O/$1_kernel_stats.csv \;
  find /tmp/p_$1 -name "*kernel_trace.csv" -exec cp {} $O/$1_kernel_trace.csv \;
  find /tmp/p_$1 -name "*memory_copy_trace.csv" -exec cp {} $O/$1_copy_trace.csv \;
  grep -h '^{' $O/prof_$1.log > $O/$1_line.json || true
}
prof c4 "--workload c4" && prof c4h2 "--workload c4h --inflight 2" && prof c4hc2 "--workload c4h --components --inflight 2"
