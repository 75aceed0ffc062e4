# GPU A/B of library variants built by tools/build_ab.sh: for each tag in $TAGS,
# swap ab_libs/<tag>/libcordahip.so in, run the GPU parity tests of $TEST
# (default: Ed25519) and a
# short C2 bench (its verdict check compares all 2^24 lanes with the corpus).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
cp $R/corda_amd/libcordahip.so $O/orig.so
for v in $TAGS; do
  cp $R/ab_libs/$v/libcordahip.so $R/corda_amd/libcordahip.so
  timeout -k 10 300 python -u -m pytest ${TEST:-tests/test_gpu_ed25519.py} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  timeout -k 10 300 python bench.py --workload ${WL:-c2} $BENCH_EXTRA --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > $O/bench_${WL:-c2}_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_${WL:-c2}_$v.json'));print('$v', round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],2), 'ms', d['verdict_check'])"
done
cp $O/orig.so $R/corda_amd/libcordahip.so
