# host-pipeline trace (c2h, c3h), then a slice of the fully oracle-checked agreement sweep
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3d
mkdir -p $O
cd $R
for wl in c2h c3h; do
  CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline > $O/trace_$wl.json 2> $O/trace_$wl.err || { echo "trace $wl failed"; tail -5 $O/trace_$wl.err; exit 1; }
  grep "cordahip" $O/trace_$wl.err | tail -12
done
timeout -k 10 ${SWEEP_S:-900} python -u tools/agree_1e9.py --oracle-all --ed ${ED:-14} --ec ${EC:-0} --first ${FIRST:-0} --threads 16 --log $O/agree_log.jsonl > $O/agree.out 2>&1; rc=$?
tail -3 $O/agree.out
exit $rc
