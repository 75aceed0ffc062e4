# r05 A/B (measurement only): CUs kept out of the Ed25519 streams -- balanced per XCD
# (CORDAHIP_AB_ED_CU_RESERVE=r: r/8 per XCD) or one whole XCD (CORDAHIP_AB_ED_XCD_RESERVE=1);
# processes alternated, c4h --components and c4h
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s2
mkdir -p $O
cd $R
for rep in 1 2; do
  for cfg in base:X=1 b16:CORDAHIP_AB_ED_CU_RESERVE=16 b32:CORDAHIP_AB_ED_CU_RESERVE=32 b48:CORDAHIP_AB_ED_CU_RESERVE=48 xcd:CORDAHIP_AB_ED_XCD_RESERVE=1; do
    t=${cfg%%:*}; ev=${cfg#*:}
    for w in comp leaves; do
      F=""; [ $w = comp ] && F=--components
      env $ev timeout -k 10 300 python -u tools/c4h_ab.py $F --rounds 3 --calls 5 dflt: > $O/${w}_${t}_$rep.json 2> $O/${w}_${t}_$rep.err || { echo "$w $t failed"; tail -20 $O/${w}_${t}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${w}_${t}_$rep.json')); v=d['sig_per_s']['dflt']; print('$w $t rep $rep', round(v['median']/1e6,2), d['check'].get('mismatches_vs_construction'), d['check'].get('txid_mismatches_vs_device_path'))"
    done
  done
done
