# Round-4 GPU call g: host-phase traces (CORDAHIP_TRACE) of c4h and c2h
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_g
mkdir -p $O
cd $R
for wl in c4h c2h; do
  CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline --no-clock > $O/$wl.json 2> $O/$wl.err || { echo "$wl failed"; tail -5 $O/$wl.err; exit 1; }
  grep cordahip $O/$wl.err | tail -24
done
