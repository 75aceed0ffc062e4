# r06: 8 signature stages (ab_libs/st8) vs 6 (the library), and three calls in
# flight, for c4h --components / c4h; alternating on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ad
mkdir -p $O
cd $R
cp corda_amd/libcordahip.so $O/base.so
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 20 --warmup 4 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
use() { cp $1 $R/corda_amd/libcordahip.so; }
for rep in 1 2; do
  use $O/base.so && run c4_$rep "--workload c4" && run hc_st6_$rep "--workload c4h --components --inflight 2" && \
  run hc_st6_if3_$rep "--workload c4h --components --inflight 3" && run h_st6_$rep "--workload c4h --inflight 2" && \
  use ab_libs/st8/libcordahip.so && run hc_st8_$rep "--workload c4h --components --inflight 2" && \
  run h_st8_$rep "--workload c4h --inflight 2" || { use $O/base.so; exit 1; }
done
use $O/base.so
