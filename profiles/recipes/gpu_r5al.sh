# r05: split Ed25519 prep for leaf signed-tx batches only -- the GPU suite, smoke, c4h lines
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5al
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for w in leaves comp c4; do
  F=""; [ $w = comp ] && F=--components; [ $w = c4 ] && F="--workload c4"
  timeout -k 10 300 python -u tools/c4h_ab.py $F --rounds 4 --calls 5 dflt: > $O/$w.json 2> $O/$w.err || { echo "$w failed"; tail -20 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); v=d['sig_per_s']['dflt']; print('$w', round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2), d['check'].get('mismatches_vs_construction'), d['check'].get('txid_mismatches_vs_device_path'))"
done
