# r05: raised wave priority of the id kernels -- parity, then A/B (CORDAHIP_ID_PRIO=0/1) on
# c4h --components (2^16 / 2^17 chunks), c4h (synthetic 838-B leaves) and c4, one box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5j
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kryo.py tests/test_gpu_txcomp.py tests/test_gpu_tx.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"
run() {  # tag, workload args, env...
  local t=$1 w=$2; shift 2
  env "$@" $B $w > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -20 $O/$t.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$t.json')); v=d['verdict_check']; print('$t', round(d['value']/1e6,2), round(d['clock']['clock_ghz'],3), v.get('mismatches_vs_construction'), v.get('txid_mismatches_vs_device_path'))"
}
run comp_p1_c16 "--workload c4h --components" X=1 && run comp_p0_c16 "--workload c4h --components" CORDAHIP_ID_PRIO=0 && \
run comp_p1_c17 "--workload c4h --components" CORDAHIP_TX_SIG_CHUNK=131072 && run comp_p0_c17 "--workload c4h --components" CORDAHIP_ID_PRIO=0 CORDAHIP_TX_SIG_CHUNK=131072 && \
run c4h_p1 "--workload c4h" X=1 && run c4h_p0 "--workload c4h" CORDAHIP_ID_PRIO=0 && run c4_p1 "--workload c4" X=1 && run c4_p0 "--workload c4" CORDAHIP_ID_PRIO=0 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/t5j -o t -- python3 $R/bench.py --workload c4h --components --steps 1 --warmup 1 --no-cpu-baseline --no-clock > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
find /tmp/t5j -name "*kernel_trace.csv" -exec cp {} $O/comp_kernel_trace.csv \;
find /tmp/t5j -name "*memory_copy_trace.csv" -exec cp {} $O/comp_memory_copy_trace.csv \;
python3 $R/tools/c4h_timeline.py $O/comp_kernel_trace.csv $O/comp_memory_copy_trace.csv > $O/timeline.txt && head -8 $O/timeline.txt
