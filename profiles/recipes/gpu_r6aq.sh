# r06: rocprofv3 kernel summaries of the final library's signed-tx lines
# (C4, C4 --device-encode, c4h / c4h --components at two calls in flight)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6aq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
prof() {
  rm -rf /tmp/p_$1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_$1 -o p -- python3 $R/bench.py $2 --no-cpu-baseline --no-clock > $O/b_$1.json 2> $O/b_$1.err || { echo "prof $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  find /tmp/p_$1 -name "*kernel_stats.csv" -exec cp {} $O/$1_kernel_stats.csv \;
  echo "$1 done"
}
prof c4 "--workload c4" && prof c4de "--workload c4 --device-encode" && \
prof c4h2 "--workload c4h --inflight 2 --steps 10 --warmup 2" && prof c4hc2 "--workload c4h --components --inflight 2 --steps 10 --warmup 2"
