# c4h: where the tx-id slices' leaf copies go (CORDAHIP_IDCOPY 0: the context
# stream, 1: a stream of their own created last, 2: ... at high priority,
# 3: ... created before the pipeline streams); c2h beside each
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3l
mkdir -p $O
cd $R
for v in ${VARS:-0 1 2 3}; do
  for wl in c4h c2h; do
    CORDAHIP_IDCOPY=$v CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_${wl}_$v.json 2> $O/trace_${wl}_$v.err || { echo "bench $wl $v failed"; tail -n 5 $O/trace_${wl}_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${wl}_$v.json'));print('$wl idcopy $v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', d['verdict_check'].get('mismatches_vs_construction'))"
  done
done
