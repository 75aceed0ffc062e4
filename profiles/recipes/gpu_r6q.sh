# r06: per-call trace of c4h --components --inflight 2 (chain type, misses, call times)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6q
mkdir -p $O
cd $R
for k in 1 2; do
CORDAHIP_TRACE=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 20 --warmup 2 --workload c4h --components --inflight 2 > $O/b$k.json 2> $O/trace$k.txt || { echo "bench failed"; tail -20 $O/trace$k.txt; exit 1; }
python3 -c "import json;d=json.load(open('$O/b$k.json'));print('value', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
grep -c "templates-only chain (" $O/trace$k.txt; grep -c "full encoder" $O/trace$k.txt; grep -c "redone" $O/trace$k.txt
grep "signed tx batch" $O/trace$k.txt | sed 's/.*done at //' | tr '\n' ' '; echo
done
