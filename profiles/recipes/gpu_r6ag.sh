# r06: kernel traces of C3 and c3h (3 steps each): per-kernel totals and the GPU's
# busy union over the timed steps (tools/trace_steady.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
tr() {
  rm -rf /tmp/t_$1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_$1 -o t -- python3 $R/bench.py $2 --no-cpu-baseline --no-clock --steps 3 --warmup 1 > $O/b_$1.json 2> $O/b_$1.err || { echo "trace $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  f=$(find /tmp/t_$1 -name "*kernel_trace.csv" | head -1)
  gzip -c $f > $O/kt_$1.csv.gz
  find /tmp/t_$1 -name "*kernel_stats.csv" -exec cp {} $O/ks_$1.csv \;
  echo "$1 done"
}
tr c3 "--workload c3" && tr c3h "--workload c3h"
