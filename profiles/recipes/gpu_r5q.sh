# r05: id slices per call (uniform CORDAHIP_TX_SLICES) x lookahead, interleaved on one corpus
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5q
mkdir -p $O
cd $R
S=CORDAHIP_TX_SLICES; A=CORDAHIP_TX_SLICE_AHEAD
timeout -k 10 300 python -u tools/c4h_ab.py --components --rounds 5 --calls 5 dflt: s10:$S=10 s6:$S=6 s10a2:$S=10,$A=2 s20a2:$S=20,$A=2 s40a3:$S=40,$A=3 > $O/comp.json 2> $O/comp.err || { echo "comp failed"; tail -20 $O/comp.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/comp.json')); print(d['check']); [print(k, round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2)) for k,v in d['sig_per_s'].items()]"
timeout -k 10 300 python -u tools/c4h_ab.py --rounds 5 --calls 5 dflt: s10:$S=10 s10a2:$S=10,$A=2 s20a2:$S=20,$A=2 > $O/leaves.json 2> $O/leaves.err || { echo "leaves failed"; tail -20 $O/leaves.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/leaves.json')); print(d['check']); [print(k, round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2)) for k,v in d['sig_per_s'].items()]"
