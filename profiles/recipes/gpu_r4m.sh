# Round-4 GPU call m: GPU suite on the two-stream host pipelines, then the
# boundary lines (c4h chunk sizes, c2h, c3h) beside their device-resident refs
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_${TAG:-m}
mkdir -p $O
cd $R
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
fi
run() {  # name, env, workload
  env $2 timeout -k 10 300 python -u bench.py --workload $3 --steps 5 --warmup 1 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$1.json'));c=d['verdict_check'];print('$1', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms clk', round(d.get('clock_ghz') or 0,3), 'mism', c.get('mismatches_vs_construction'), c.get('mismatches_vs_oracle_open_lanes'), c.get('txid_mismatches_vs_device_path'), c.get('verdict_word_mismatches'))"
}
for c in ${CHUNKS:-65536 131072 262144}; do run c4h_$c CORDAHIP_TX_SIG_CHUNK=$c c4h || exit 1; done
for w in ${WLS:-c4 c2h c2 c3h c3}; do run $w X=1 $w || exit 1; done
