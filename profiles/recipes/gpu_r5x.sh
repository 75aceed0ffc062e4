# r05: SHA-256 midstates of the templates' all-constant blocks -- parity, then c4h --components
# with C4 on the same box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5x
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kryo.py tests/test_gpu_txcomp.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for w in comp c4 comp; do
  F="--components"; [ $w = c4 ] && F="--workload c4"
  timeout -k 10 300 python -u tools/c4h_ab.py $F --rounds 4 --calls 5 dflt: > $O/$w.json 2> $O/$w.err || { echo "$w failed"; tail -20 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); v=d['sig_per_s']['dflt']; print('$w', round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2), d['check'].get('mismatches_vs_construction'), d['check'].get('txid_mismatches_vs_device_path'))"
done
