# r05 A/B (measurement only): leaf hashes from the templates (kryo_hash, descriptors a block
# ahead) against template writes + sha256_leaves in the templates-only chain, interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5w
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_txcomp.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/c4h_ab.py --components --rounds 6 --calls 5 fused: write:CORDAHIP_AB_FUSED_HASH=0 > $O/comp.json 2> $O/comp.err || { echo "comp failed"; tail -20 $O/comp.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/comp.json')); print(d['check'].get('mismatches_vs_construction'), d['check'].get('txid_mismatches_vs_device_path')); [print(k, round(v['median']/1e6,2), round(v['min']/1e6,2), round(v['max']/1e6,2)) for k,v in d['sig_per_s'].items()]"
