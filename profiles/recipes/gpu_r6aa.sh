# r06: pinned signature stages per transaction set (3 = base, 4, 5, 6; ab_libs/st<N>)
# for c4h / c4h --components at --inflight 2, alternating libraries on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6aa}
mkdir -p $O
cd $R
cp corda_amd/libcordahip.so $O/base.so
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 20 --warmup 4 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
use() { cp $1 $R/corda_amd/libcordahip.so; }
HC="--workload c4h --components --inflight 2"
H="--workload c4h --inflight 2"
for rep in 1 2; do
  use $O/base.so && run hc_st3_$rep "$HC" && use ab_libs/st4/libcordahip.so && run hc_st4_$rep "$HC" && \
  use ab_libs/st5/libcordahip.so && run hc_st5_$rep "$HC" && use ab_libs/st6/libcordahip.so && run hc_st6_$rep "$HC" && \
  use $O/base.so && run h_st3_$rep "$H" && use ab_libs/st5/libcordahip.so && run h_st5_$rep "$H" && \
  use ab_libs/st6/libcordahip.so && run h_st6_$rep "$H" || { use $O/base.so; exit 1; }
done
use $O/base.so
