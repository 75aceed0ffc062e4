# r05: kernel + copy trace of c4h --components (one warm call) for tools/c4h_timeline.py
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in comp leaves; do
  F=--components; [ $w = leaves ] && F=--native-leaves
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/t5e_$w -o t -- python3 $R/bench.py --workload c4h $F --steps 1 --warmup 1 --no-cpu-baseline --no-clock > $O/trace_$w.log 2>&1 || { echo "trace $w failed"; tail -20 $O/trace_$w.log; exit 1; }
  find /tmp/t5e_$w -name "*kernel_trace.csv" -exec cp {} $O/${w}_kernel_trace.csv \;
  find /tmp/t5e_$w -name "*memory_copy_trace.csv" -exec cp {} $O/${w}_memory_copy_trace.csv \;
  python3 $R/tools/c4h_timeline.py $O/${w}_kernel_trace.csv $O/${w}_memory_copy_trace.csv > $O/timeline_$w.txt && cat $O/timeline_$w.txt
done
cd $R
B="timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"
$B --workload c4 > $O/c4.json 2> $O/c4.err && $B --workload c4h > $O/c4h.json 2> $O/c4h.err && python3 -c "
import json
for f in ('c4','c4h'):
    d=json.load(open('$O/'+f+'.json')); print(f, round(d['value']/1e6,2), d['clock']['clock_ghz'])"
