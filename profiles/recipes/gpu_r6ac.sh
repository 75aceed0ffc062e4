# r06: the whole GPU suite on the current library (six signature stages per
# transaction set), then c4, c4h and c4h --components at --inflight 2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ac
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|passed|failed" $O/pytest_gpu.log | tail -20; exit 1; }
tail -1 $O/pytest_gpu.log
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 20 --warmup 4 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), d.get('device_mem_gb'), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
for rep in 1 2; do
  run c4_$rep "--workload c4" && run h_$rep "--workload c4h --inflight 2" && run hc_$rep "--workload c4h --components --inflight 2" || exit 1
done
