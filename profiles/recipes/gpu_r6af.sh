# r06: c3h host chunk size (CORDAHIP_HOST_CHUNK 2^22 default, 2^23, 2^24) against C3,
# alternating on one box: are the ECDSA chunks' end-of-grid tails (one ECDSA stream,
# one workspace) the c3h gap?
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6af
mkdir -p $O
cd $R
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 3 --warmup 1 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
for rep in 1 2; do
  run c3_$rep "--workload c3" && run c3h_22_$rep "--workload c3h" && CORDAHIP_HOST_CHUNK=8388608 run c3h_23_$rep "--workload c3h" && \
  CORDAHIP_HOST_CHUNK=16777216 run c3h_24_$rep "--workload c3h" || exit 1
done
