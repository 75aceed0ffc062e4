# r05 A/B: geometric tail of the signature chunks (CORDAHIP_TX_SIG_TAIL_MIN) and a smaller
# first chunk, interleaved on one corpus, c4h and c4h --components; C4 alongside
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5t
mkdir -p $O
cd $R
T=CORDAHIP_TX_SIG_TAIL_MIN; K=CORDAHIP_TX_SIG_CHUNK; M=CORDAHIP_TX_SIG_CHUNK_MAX
for w in leaves comp; do
  F=""; [ $w = comp ] && F=--components
  timeout -k 10 300 python -u tools/c4h_ab.py $F --rounds 6 --calls 5 dflt: t16:$T=16384 t32:$T=32768 t16r:$T=16384,$K=32768,$M=131072 r15:$K=32768,$M=131072 > $O/$w.json 2> $O/$w.err || { echo "$w failed"; tail -20 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', d['check'].get('mismatches_vs_construction'), d['check'].get('txid_mismatches_vs_device_path')); [print(k, round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2)) for k,v in d['sig_per_s'].items()]"
done
timeout -k 10 300 python -u tools/c4h_ab.py --workload c4 --rounds 6 --calls 5 dflt: > $O/c4.json 2> $O/c4.err && python3 -c "import json; d=json.load(open('$O/c4.json')); print('c4', round(d['sig_per_s']['dflt']['median']/1e6,2))"
