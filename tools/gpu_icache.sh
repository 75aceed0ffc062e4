# Instruction-cache counters of the hot kernels (one rocprofv3 --pmc pass per
# group, each under its own KILL timeout): WL (c2|c3), LOG2 batch size.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/icache_${TAG:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --workload ${WL:-c2} --batch-log2 ${LOG2:-22} --steps 1 --warmup 0 --no-cpu-baseline"
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_VALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d /tmp/icache_$i -o p -- $BENCH > $O/pass$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
  find /tmp/icache_$i -name "*counter_collection.csv" -exec cp {} $O/pass$i.csv \;
done
python3 $R/tools/pmc_summary.py $O/pass*.csv > $O/summary.json && python3 - <<PY
import json
d=json.load(open("$O/summary.json"))
for k,v in d.items():
    if any(s in k for s in ("sign","gtable","btable")): continue
    h,m=v.get("SQC_ICACHE_HITS",0),v.get("SQC_ICACHE_MISSES",0)
    print(k[:60], "hits",h,"misses",m,"miss%%", round(100*m/max(h+m,1),2), "ifetch",v.get("SQ_IFETCH"), "valu",v.get("SQ_INSTS_VALU"))
PY
