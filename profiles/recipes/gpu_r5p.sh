# r05: kernel + copy trace of c4h --components with the current defaults (2^17 chunks, id priority,
# templates-only chain)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/t5p -o t -- python3 $R/bench.py --workload c4h --components --steps 1 --warmup 1 --no-cpu-baseline --no-clock > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
find /tmp/t5p -name "*kernel_trace.csv" -exec cp {} $O/comp_kernel_trace.csv \;
find /tmp/t5p -name "*memory_copy_trace.csv" -exec cp {} $O/comp_memory_copy_trace.csv \;
python3 $R/tools/c4h_timeline.py $O/comp_kernel_trace.csv $O/comp_memory_copy_trace.csv > $O/timeline.txt && head -8 $O/timeline.txt
# and the encoder kernels' instruction / TA counters (as tools/gpu_r5c.sh, on the current writer)
K="python3 $R/tools/kryo_dev_bench.py --txs 262144 --calls 2"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" "TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TCC_WRITE_REQ TCP_TCC_READ_REQ"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc5p_$i -o p -- $K > $O/pass$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
  find /tmp/pmc5p_$i -name "*counter_collection.csv" -exec cp {} $O/pass$i.csv \;
done
python3 $R/tools/pmc_summary.py $O/pass*.csv > $O/summary.json && python3 -c "
import json; s=json.load(open('$O/summary.json'))
for k,v in s.items():
    if 'kryo' in k: print(k[:60], {a: round(b) for a,b in v.items()})"
