# r05: twrite with the constant copy loaded beside its descriptor -- parity, encoder alone x3
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5aa
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kryo.py tests/test_gpu_txcomp.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for k in 1 2 3; do
  timeout -k 10 200 python tools/kryo_dev_bench.py > $O/kdb$k.json 2> $O/kdb$k.err || { echo "kdb failed"; tail $O/kdb$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/kdb$k.json')); print('encoder ms', round(d['ms_median'],3), d['leaves_equal_host'], d['item_errors'])"
done
