# r05: fused merkle (+ component check + host stores), no counter reset in the templates-only
# chain, records compared from LDS -- parity, encoder alone, c4h lines, c4h --components trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5r
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kryo.py tests/test_gpu_txcomp.py tests/test_gpu_tx.py tests/test_gpu_multidevice.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/kryo_dev_bench.py > $O/kdb.json 2> $O/kdb.err || { echo "kdb failed"; tail $O/kdb.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/kdb.json')); print('encoder ms', round(d['ms_median'],3), d['leaves_equal_host'], d['item_errors'])"
timeout -k 10 300 python -u tools/c4h_ab.py --components --rounds 4 --calls 5 dflt: > $O/comp.json 2> $O/comp.err || { echo "comp failed"; tail -20 $O/comp.err; exit 1; }
timeout -k 10 300 python -u tools/c4h_ab.py --rounds 4 --calls 5 dflt: > $O/leaves.json 2> $O/leaves.err || { echo "leaves failed"; tail -20 $O/leaves.err; exit 1; }
timeout -k 10 300 python -u tools/c4h_ab.py --workload c4 --rounds 4 --calls 5 dflt: > $O/c4.json 2> $O/c4.err || { echo "c4 failed"; tail -20 $O/c4.err; exit 1; }
python3 -c "
import json
for f in ('comp','leaves','c4'):
    d=json.load(open('$O/'+f+'.json')); v=d['sig_per_s']['dflt']; print(f, round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2), d['check'].get('mismatches_vs_construction'), d['check'].get('txid_mismatches_vs_device_path'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/t5r -o t -- python3 $R/bench.py --workload c4h --components --steps 1 --warmup 1 --no-cpu-baseline --no-clock > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
find /tmp/t5r -name "*kernel_trace.csv" -exec cp {} $O/comp_kernel_trace.csv \;
find /tmp/t5r -name "*memory_copy_trace.csv" -exec cp {} $O/comp_memory_copy_trace.csv \;
python3 $R/tools/c4h_timeline.py $O/comp_kernel_trace.csv $O/comp_memory_copy_trace.csv > $O/timeline.txt && head -3 $O/timeline.txt
