# r05: shape pass with block-sized tiles and one table probe per wave per hash -- parity,
# the encoder alone, its fabric bytes (FETCH_SIZE / WRITE_SIZE), then c4h --components and c4de
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5n
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kryo.py tests/test_gpu_txcomp.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/kryo_dev_bench.py > $O/kdb.json 2> $O/kdb.err || { echo "kdb failed"; tail $O/kdb.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/kdb.json')); print('encoder ms', round(d['ms_median'],3), d['leaves_equal_host'], d['item_errors'])"
cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/kryo_dev_bench.py --txs 262144 --calls 2"
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc5n_$i -o p -- $K > $O/pass$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
  find /tmp/pmc5n_$i -name "*counter_collection.csv" -exec cp {} $O/pass$i.csv \;
done
python3 $R/tools/pmc_kryo_traffic.py $O/pass1.csv $O/pass2.csv 262144 3 > $O/r05_pmc_kryo_traffic.json && python3 -c "
import json; s=json.load(open('$O/r05_pmc_kryo_traffic.json')); print(round(s['l2_fabric_bytes_per_tx']), {k: (round(v['fetch_bytes_per_tx']), round(v['write_bytes_per_tx'])) for k,v in s['kernels'].items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p5n -o kdb -- python3 $R/tools/kryo_dev_bench.py > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
find /tmp/p5n -name "*kernel_stats.csv" -exec cp {} $O/kdb_kernel_stats.csv \;
cd $R
B="timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline"
$B --workload c4h --components > $O/c4hc.json 2> $O/c4hc.err || { echo "c4hc failed"; tail -20 $O/c4hc.err; exit 1; }
$B --workload c4 --device-encode > $O/c4de.json 2> $O/c4de.err || { echo "c4de failed"; tail -20 $O/c4de.err; exit 1; }
python3 -c "
import json
for f in ('c4hc','c4de'):
    d=json.load(open('$O/'+f+'.json')); print(f, round(d['value']/1e6,2), round(d['clock']['clock_ghz'],3), d['verdict_check'])"
