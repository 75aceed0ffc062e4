# Round-4 GPU call l: c4h chunk-size A/B on one box (CORDAHIP_TX_SIG_CHUNK: first chunk C, then 2C)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_l
mkdir -p $O
cd $R
for c in 131072 65536 262144 131072; do
  CORDAHIP_TX_SIG_CHUNK=$c timeout -k 10 300 python -u bench.py --workload c4h --steps 5 --warmup 1 --no-cpu-baseline > $O/c4h_$c.json 2> $O/c4h_$c.err || { echo "c4h $c failed"; tail -5 $O/c4h_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c4h_$c.json'));print('c4h chunk $c', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms clk', round(d.get('clock_ghz') or 0,3), d['verdict_check'])"
done
timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { echo "c4 failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/c4.json'));print('c4', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms clk', round(d.get('clock_ghz') or 0,3))"
