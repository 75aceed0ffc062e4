# r05: leaf hashes straight from the templates in the templates-only chain -- parity, then
# c4h --components / c4h / C4 interleaved lines
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5v
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kryo.py tests/test_gpu_txcomp.py tests/test_gpu_tx.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for w in comp leaves c4; do
  F=""; [ $w = comp ] && F=--components; [ $w = c4 ] && F="--workload c4"
  timeout -k 10 300 python -u tools/c4h_ab.py $F --rounds 4 --calls 5 dflt: > $O/$w.json 2> $O/$w.err || { echo "$w failed"; tail -20 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); v=d['sig_per_s']['dflt']; print('$w', round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2), d['check'].get('mismatches_vs_construction'), d['check'].get('txid_mismatches_vs_device_path'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/t5v -o t -- python3 $R/bench.py --workload c4h --components --steps 1 --warmup 1 --no-cpu-baseline --no-clock > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
find /tmp/t5v -name "*kernel_trace.csv" -exec cp {} $O/comp_kernel_trace.csv \;
find /tmp/t5v -name "*memory_copy_trace.csv" -exec cp {} $O/comp_memory_copy_trace.csv \;
python3 $R/tools/c4h_timeline.py $O/comp_kernel_trace.csv $O/comp_memory_copy_trace.csv > $O/timeline.txt && head -3 $O/timeline.txt
