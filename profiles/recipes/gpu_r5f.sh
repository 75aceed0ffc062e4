# r05: after the tile-local shape mapping, small fallback grids and the tx-major corpus:
# parity, the encoder alone, c4h --components (lookahead 1..3) and its trace, fabric bytes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5f
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kryo.py tests/test_gpu_txcomp.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/kryo_dev_bench.py > $O/kdb.json 2> $O/kdb.err || { echo "kdb failed"; tail $O/kdb.err; exit 1; }
cat $O/kdb.json
B="timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"
for a in 1 2 3; do
  CORDAHIP_TX_SLICE_AHEAD=$a $B --workload c4h --components > $O/c4hc_a$a.json 2> $O/c4hc_a$a.err || { echo "c4hc $a failed"; tail -20 $O/c4hc_a$a.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4hc_a$a.json')); print('ahead $a', round(d['value']/1e6,2), d['clock']['clock_ghz'], d['verdict_check'])"
done
$B --workload c4 --device-encode > $O/c4de.json 2> $O/c4de.err || { echo "c4de failed"; tail -20 $O/c4de.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c4de.json')); print('c4de', round(d['value']/1e6,2), d['clock']['clock_ghz'], d['verdict_check'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/t5f -o t -- python3 $R/bench.py --workload c4h --components --steps 1 --warmup 1 --no-cpu-baseline --no-clock > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
find /tmp/t5f -name "*kernel_trace.csv" -exec cp {} $O/comp_kernel_trace.csv \;
find /tmp/t5f -name "*memory_copy_trace.csv" -exec cp {} $O/comp_memory_copy_trace.csv \;
python3 $R/tools/c4h_timeline.py $O/comp_kernel_trace.csv $O/comp_memory_copy_trace.csv > $O/timeline.txt && cat $O/timeline.txt
K="python3 $R/tools/kryo_dev_bench.py --txs 262144 --calls 2"
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc5f_$i -o p -- $K > $O/pass$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
  find /tmp/pmc5f_$i -name "*counter_collection.csv" -exec cp {} $O/pass$i.csv \;
done
python3 $R/tools/pmc_kryo_traffic.py $O/pass1.csv $O/pass2.csv 262144 3 > $O/r05_pmc_kryo_traffic.json && python3 -c "
import json; s=json.load(open('$O/r05_pmc_kryo_traffic.json')); print(s['l2_fabric_bytes_per_tx'], {k: round(v['fetch_bytes_per_tx']+v['write_bytes_per_tx']) for k,v in s['kernels'].items()})"
