# Round-4 scoreboard on the committed tree for the workloads final5/final6 did
# not cover: C1 (the reference's CPU-runnable case), C3, c3h, c4 --device-encode.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_final8
mkdir -p $O
cd $R
run() {  # name, workload args
  timeout -k 10 400 python -u bench.py $2 > $O/bench_$1.json 2> $O/bench_$1.err || { echo "$1 failed"; tail -8 $O/bench_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$1.json'));print('$1', round(d['value']/1e6,2), 'M/s', d['roofline']['frac'], d['verdict_check'])"
}
run c1 "--workload c1" || exit 1
run c3 "--workload c3" || exit 1
run c3h "--workload c3h" || exit 1
run c4_devenc "--workload c4 --device-encode --no-cpu-baseline" || exit 1
