set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1b
P=/tmp/prof_r1b
mkdir -p $O $P
cd $R
if [ -z "$SKIP_PYTEST" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
fi
WL=${WL:-c2 c3 c4}
for w in $WL; do
  timeout -k 10 600 python bench.py --workload $w --steps 3 --warmup 1 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -20 $O/bench_$w.err; exit 1; }
  echo "bench $w ok"
done
cd /tmp && export TMPDIR=/tmp
for w in $WL; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/$w -o $w -- python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_$w.log 2>&1 || { echo "prof $w failed"; tail -20 $O/prof_$w.log; exit 1; }
  find $P/$w -name "*stats*" -exec cp {} $O/ \;
done
ls -la $O
echo done
