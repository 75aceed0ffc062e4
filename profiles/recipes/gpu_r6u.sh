# r06 (second A/B, no tests): device signed-tx calls with the Ed25519 section in alternating 2^k-signature
# chunks (CORDAHIP_DEVICE_ED_CHUNK; 0 = one launch pair) -- device-path tests, then
# c4 and c4 --device-encode A/B, alternating, one box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6u
mkdir -p $O
cd $R
true
true
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 10 --warmup 2 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
for rep in 1 2; do
  CORDAHIP_DEVICE_ED_CHUNK=65536 run c4_c16_$rep "--workload c4" && CORDAHIP_DEVICE_ED_CHUNK=131072 run c4_c17_$rep "--workload c4" && \
  CORDAHIP_DEVICE_ED_CHUNK=98304 run c4_c1615_$rep "--workload c4" && CORDAHIP_DEVICE_ED_CHUNK=32768 run c4_c15_$rep "--workload c4" && \
  CORDAHIP_DEVICE_ED_CHUNK=65536 run de_c16_$rep "--workload c4 --device-encode" && CORDAHIP_DEVICE_ED_CHUNK=131072 run de_c17_$rep "--workload c4 --device-encode" && \
  CORDAHIP_DEVICE_ED_CHUNK=98304 run de_c1615_$rep "--workload c4 --device-encode" || exit 1
done
