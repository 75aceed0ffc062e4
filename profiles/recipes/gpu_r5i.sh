# r05: the templates-only component chain -- parity (kryo + txcomp GPU tests), then
# c4h --components at 2^16 / 2^17 signature chunks, the full chain forced for comparison
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5i
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kryo.py tests/test_gpu_txcomp.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --workload c4h --components"
run() {  # tag, env...
  local t=$1; shift
  env "$@" $B > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -20 $O/$t.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$t.json')); v=d['verdict_check']; print('$t', round(d['value']/1e6,2), round(d['clock']['clock_ghz'],3), v['mismatches_vs_construction'], v['txid_mismatches_vs_device_path'])"
}
run tpl_c16 X=1 && run tpl_c17 CORDAHIP_TX_SIG_CHUNK=131072 && run full_c17 CORDAHIP_TX_SIG_CHUNK=131072 CORDAHIP_KRYO_TEMPLATES_ONLY=0 && run tpl_c17_a2 CORDAHIP_TX_SIG_CHUNK=131072 CORDAHIP_TX_SLICE_AHEAD=2
