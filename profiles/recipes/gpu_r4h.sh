# Round-4 GPU call h: is the host pipeline throttled by the box's CPU quota?
# cgroup cpu.stat around c4h / c2h runs at 16 and 8 host packing threads
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_h
mkdir -p $O
cd $R
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc
for th in 16 8; do
  for wl in c4h c2h; do
    s0=$(grep throttled_usec /sys/fs/cgroup/cpu.stat 2>/dev/null | head -1)
    CORDAHIP_HOST_THREADS=$th CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload $wl --steps 4 --warmup 1 --no-cpu-baseline --no-clock > $O/${wl}_$th.json 2> $O/${wl}_$th.err || { echo "$wl failed"; tail -5 $O/${wl}_$th.err; exit 1; }
    s1=$(grep throttled_usec /sys/fs/cgroup/cpu.stat 2>/dev/null | head -1)
    python3 -c "import json;d=json.load(open('$O/${wl}_$th.json'));print('$wl threads $th', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms')"
    echo "  throttle before: $s0 after: $s1"
    grep -c "launch [0-9][0-9]*\.[0-9]* ms" $O/${wl}_$th.err > /dev/null
    grep cordahip $O/${wl}_$th.err | awk '{for(i=1;i<=NF;i++) if($i=="launch" && $(i+1)+0>2) print "  slow launch:", $0}' | tail -4
  done
done
