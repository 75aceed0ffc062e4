# r06: generic signature batches (cordahip_sig_submit) with two calls outstanding:
# c2h / c3h at --inflight 1 and 2 against C2 / C3, alternating on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ah
mkdir -p $O
cd $R
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 8 --warmup 2 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), d.get('device_mem_gb', {}).get('peak'), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k and v})"
}
for rep in 1 2; do
  run c3_$rep "--workload c3" && run c3h1_$rep "--workload c3h" && run c3h2_$rep "--workload c3h --inflight 2" && \
  run c2_$rep "--workload c2" && run c2h1_$rep "--workload c2h" && run c2h2_$rep "--workload c2h --inflight 2" || exit 1
done
