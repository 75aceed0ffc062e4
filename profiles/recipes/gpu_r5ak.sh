# r05 A/B (measurement only): the Ed25519 prep split (keys/R first, the ids' gather and the
# message half after) against the fused prep, in the signed-tx chunks; parity first
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ak
mkdir -p $O
cd $R
true

for w in leaves comp; do
  F=""; [ $w = comp ] && F=--components
  timeout -k 10 300 python -u tools/c4h_ab.py $F --rounds 10 --calls 5 split: fused:CORDAHIP_AB_NO_SPLIT=1 > $O/$w.json 2> $O/$w.err || { echo "$w failed"; tail -20 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', d['check'].get('mismatches_vs_construction'), d['check'].get('txid_mismatches_vs_device_path')); [print(k, round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2)) for k,v in d['sig_per_s'].items()]"
done
