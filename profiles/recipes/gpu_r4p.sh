# Round-4 GPU call p: tx tests, then bench lines given as RUNS="name|ENV=..|workload ..."
# (default: c4h default / c4h 2^15 first chunks / C4 / c2h / C2), one traced c4h
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_${TAG:-p}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_tx.py tests/test_gpu_multidevice.py tests/test_gpu_host_batch.py} -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
run() {  # name, env, workload
  env $2 timeout -k 10 300 python -u bench.py --workload $3 --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$1.json'));c=d['verdict_check'];print('$1', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms clk', round(d.get('clock_ghz') or 0,3), 'mism', c.get('mismatches_vs_construction'), c.get('txid_mismatches_vs_device_path'), c.get('mismatches_vs_oracle_open_lanes'))"
}
for spec in ${RUNS:-"c4h|X=1|c4h" "c4h_32k|CORDAHIP_TX_SIG_CHUNK=32768|c4h" "c4|X=1|c4" "c2h|X=1|c2h" "c2|X=1|c2"}; do
  IFS='|' read -r n e w <<< "$spec"
  run $n "$(echo "$e" | tr "+" " ")" $w || exit 1
done
if [ -z "$NOTRACE" ]; then
CORDAHIP_TRACE=1 timeout -k 10 300 python -u bench.py --workload c4h --steps 3 --warmup 1 --no-cpu-baseline --no-clock > $O/c4h_traced.json 2> $O/c4h_traced.err || { echo "traced failed"; exit 1; }
grep "signed tx batch" $O/c4h_traced.err | tail -3
fi
