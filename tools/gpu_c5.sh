# C5 streaming drain: GPU stream tests, then the C5 bench line + rocprof kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c5
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 200 > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python bench.py --workload c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench failed"; tail -20 $O/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c5.json')); print(d['value'], d['ms_per_step'], d['verdict_check'], d.get('cpu_baseline',{}).get('value'))"
TAG=c5 WL=c5 bash tools/gpu_prof.sh
