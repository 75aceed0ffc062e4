# r05: interleaved chunk x lookahead A/B (tools/c4h_ab.py) on one corpus per workload
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5l
mkdir -p $O
cd $R
K=CORDAHIP_TX_SIG_CHUNK; A=CORDAHIP_TX_SLICE_AHEAD
timeout -k 10 300 python -u tools/c4h_ab.py --components --rounds 6 --calls 5 c16a1: c17a1:$K=131072 c16a2:$A=2 c17a2:$K=131072,$A=2 c16a0:$A=0 c17a0:$K=131072,$A=0 c18a1:$K=262144 > $O/comp.json 2> $O/comp.err || { echo "comp failed"; tail -20 $O/comp.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/comp.json')); print(d['check']); [print(k, round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2)) for k,v in d['sig_per_s'].items()]"
timeout -k 10 300 python -u tools/c4h_ab.py --rounds 6 --calls 5 c16a1: c17a1:$K=131072 c16a2:$A=2 c16a0:$A=0 c16to17:$K=65536,CORDAHIP_TX_SIG_CHUNK_MAX=131072 > $O/leaves.json 2> $O/leaves.err || { echo "leaves failed"; tail -20 $O/leaves.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/leaves.json')); print(d['check']); [print(k, round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2)) for k,v in d['sig_per_s'].items()]"
