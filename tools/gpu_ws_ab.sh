# A/B of the Ed25519 prep/ladder launch-pair size (CORDAHIP_ED25519_WS_LANES) on C2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wsab
mkdir -p $O
cd $R
for L in ${SIZES:-262144 1048576 4194304 16777216}; do
  CORDAHIP_ED25519_WS_LANES=$L timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > $O/c2_$L.json 2> $O/c2_$L.err || { echo "bench $L failed"; tail -5 $O/c2_$L.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_$L.json')); print($L, round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],1))"
done
