# r05: shape pass staged through LDS (coalesced item loads and output stores) -- parity, encoder, lines
# encoder alone (rocprof stats), c4h --components and C4
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5z
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kryo.py tests/test_gpu_txcomp.py tests/test_gpu_tx.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/kryo_dev_bench.py > $O/kdb.json 2> $O/kdb.err || { echo "kdb failed"; tail $O/kdb.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/kdb.json')); print('encoder ms', round(d['ms_median'],3), d['leaves_equal_host'], d['item_errors'])"
for w in comp c4; do
  F="--components"; [ $w = c4 ] && F="--workload c4"
  timeout -k 10 300 python -u tools/c4h_ab.py $F --rounds 4 --calls 5 dflt: > $O/$w.json 2> $O/$w.err || { echo "$w failed"; tail -20 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); v=d['sig_per_s']['dflt']; print('$w', round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2), d['check'].get('mismatches_vs_construction'), d['check'].get('txid_mismatches_vs_device_path'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p5z -o kdb -- python3 $R/tools/kryo_dev_bench.py > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
find /tmp/p5z -name "*kernel_stats.csv" -exec cp {} $O/kdb_kernel_stats.csv \;
python3 -c "
import csv
r=list(csv.DictReader(open('$O/kdb_kernel_stats.csv')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:4]: print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1))"
