# r05: the C4 lines after the encoder rework -- device-encode C4, c4h over leaves and over
# components (cordahip_txcomp_submit), their kernel stats, the encoder's fabric bytes
# (FETCH_SIZE / WRITE_SIZE passes over tools/kryo_dev_bench.py), and the host packing
# microbench on the box's CPU share
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5d
mkdir -p $O
cd $R
B="timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"
$B --workload c4 --device-encode > $O/c4de.json 2> $O/c4de.err || { echo "c4de failed"; tail -20 $O/c4de.err; exit 1; }
cat $O/c4de.json
$B --workload c4h --components > $O/c4h_comp.json 2> $O/c4h_comp.err || { echo "c4h comp failed"; tail -20 $O/c4h_comp.err; exit 1; }
cat $O/c4h_comp.json
$B --workload c4h --native-leaves > $O/c4h_leaves.json 2> $O/c4h_leaves.err || { echo "c4h leaves failed"; tail -20 $O/c4h_leaves.err; exit 1; }
cat $O/c4h_leaves.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p5d -o c4hc -- python3 $R/bench.py --workload c4h --components --steps 2 --warmup 1 --no-cpu-baseline --no-clock > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
find /tmp/p5d -name "*kernel_stats.csv" -exec cp {} $O/c4h_comp_kernel_stats.csv \;
K="python3 $R/tools/kryo_dev_bench.py --txs 262144 --calls 2"
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc5d_$i -o p -- $K > $O/pass$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
  find /tmp/pmc5d_$i -name "*counter_collection.csv" -exec cp {} $O/pass$i.csv \;
done
python3 $R/tools/pmc_kryo_traffic.py $O/pass1.csv $O/pass2.csv 262144 3 > $O/r05_pmc_kryo_traffic.json && python3 -c "
import json; s=json.load(open('$O/r05_pmc_kryo_traffic.json')); print(s['l2_fabric_bytes_per_tx'], {k: round(v['fetch_bytes_per_tx']+v['write_bytes_per_tx']) for k,v in s['kernels'].items()})"
g++ -O2 -std=c++17 -pthread -I$R/include -o /tmp/pack_bench $R/tools/pack_bench.cpp && timeout -k 10 200 /tmp/pack_bench 4194304 16 > $O/pack_bench.jsonl && cat $O/pack_bench.jsonl
