# ECDSA A/B: full GPU test suite on the default path, then C3 bench with the affine pass fused into the ladder vs separate, + rocprof
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ecab
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in fused kernel; do
  CORDAHIP_ECDSA_AFFINE=$v timeout -k 10 500 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -20 $O/bench_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['roofline']['kernel_ms'], d['verdict_check'])"
done
LADDER=split-half TAG=ec WL=c3 bash tools/gpu_prof.sh
