# A/B of the ECDSA prep/inv/affine/ladder launch size (CORDAHIP_ECDSA_WS_SLOTS) on C3
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ecwsab
mkdir -p $O
cd $R
for L in ${SIZES:-1048576 4194304}; do
  CORDAHIP_ECDSA_WS_SLOTS=$L timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > $O/c3_$L.json 2> $O/c3_$L.err || { echo "bench $L failed"; tail -5 $O/c3_$L.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c3_$L.json')); print('c3', $L, round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],1))"
done
