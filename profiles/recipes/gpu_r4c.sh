# Round-4 GPU call c: GPU suite on the device-id tx pipeline + copy-group host
# pipeline, then before/after lines of the boundary workloads on ONE box:
# ab_libs/r4before (b736408: host-side id round trip, 2^22 chunks) vs the tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_${TAG:-c}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
cp corda_amd/libcordahip.so $O/after.so
for wl in ${WLS:-c2h c4h}; do
  for v in before after; do
    if [ $v = before ]; then cp ab_libs/r4before/libcordahip.so corda_amd/libcordahip.so; else cp $O/after.so corda_amd/libcordahip.so; fi
    timeout -k 10 420 python -u bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_${wl}_$v.json 2> $O/bench_${wl}_$v.err || { echo "bench $wl $v failed"; tail -20 $O/bench_${wl}_$v.err; cp $O/after.so corda_amd/libcordahip.so; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${wl}_$v.json'));c=d['verdict_check'];print('$wl $v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms clk', round(d.get('clock_ghz') or 0,3), 'mism', c.get('mismatches_vs_construction'), c.get('mismatches_vs_oracle_open_lanes'), c.get('txid_mismatches_vs_device_path'), c.get('verdict_word_mismatches'), 'lanes', c.get('lanes_checked'))"
  done
done
cp $O/after.so corda_amd/libcordahip.so
for wl in ${REF:-c2 c4}; do
  timeout -k 10 420 python -u bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo "bench $wl failed"; tail -20 $O/bench_$wl.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$wl.json'));print('$wl', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms clk', round(d.get('clock_ghz') or 0,3))"
done
