# r05 A/B (measurement only): c4h --components with the encoder's rare-path kernels
# (build / dsize / dwrite) skipped after the first call, and 2^17-signature chunks
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5h
mkdir -p $O
cd $R
B="timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --workload c4h --components"
run() {  # tag, env...
  local t=$1; shift
  env "$@" $B > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -20 $O/$t.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$t.json')); v=d['verdict_check']; print('$t', round(d['value']/1e6,2), round(d['clock']['clock_ghz'],3), v['mismatches_vs_construction'], v['txid_mismatches_vs_device_path'])"
}
run base X=1 && run skip CORDAHIP_AB_SKIP_RARE=1 && run skip_c17 CORDAHIP_AB_SKIP_RARE=1 CORDAHIP_TX_SIG_CHUNK=131072 && run base_c17 CORDAHIP_TX_SIG_CHUNK=131072 || exit 1
cd /tmp && export TMPDIR=/tmp
CORDAHIP_AB_SKIP_RARE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/t5h -o t -- python3 $R/bench.py --workload c4h --components --steps 1 --warmup 1 --no-cpu-baseline --no-clock > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
find /tmp/t5h -name "*kernel_trace.csv" -exec cp {} $O/comp_kernel_trace.csv \;
find /tmp/t5h -name "*memory_copy_trace.csv" -exec cp {} $O/comp_memory_copy_trace.csv \;
python3 $R/tools/c4h_timeline.py $O/comp_kernel_trace.csv $O/comp_memory_copy_trace.csv > $O/timeline.txt && cat $O/timeline.txt
