# A/B of the Ed25519 kernel variants: parity tests + C2 bench per variant
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
for v in ${VARIANTS:-split-half split}; do
  CORDAHIP_ED25519_LADDER=$v timeout -k 10 600 python -m pytest tests/test_gpu_ed25519.py tests/test_gpu_tx.py -m gpu -x -q > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
  CORDAHIP_ED25519_LADDER=$v timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -20 $O/bench_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['roofline']['kernel_ms'], d['verdict_check'])"
done
