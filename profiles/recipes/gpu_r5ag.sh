# r05: tx_of filled chunk by chunk -- parity (tx, txcomp, multidevice), then c4h / c4h --components /
# C4 interleaved lines and a host trace of one c4h call
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ag
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tx.py tests/test_gpu_txcomp.py tests/test_gpu_multidevice.py tests/test_gpu_runtime.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for w in leaves comp c4; do
  F=""; [ $w = comp ] && F=--components; [ $w = c4 ] && F="--workload c4"
  timeout -k 10 300 python -u tools/c4h_ab.py $F --rounds 4 --calls 5 dflt: > $O/$w.json 2> $O/$w.err || { echo "$w failed"; tail -20 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); v=d['sig_per_s']['dflt']; print('$w', round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2), d['check'].get('mismatches_vs_construction'), d['check'].get('txid_mismatches_vs_device_path'))"
done
CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload c4h --steps 2 --warmup 1 --no-cpu-baseline --no-clock > $O/c4h.json 2> $O/c4h_trace.err && tail -2 $O/c4h_trace.err
