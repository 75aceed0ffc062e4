# r06: kernel traces of c4h --components and c4h at --inflight 2 and of c4 (steady
# state occupancy: tools/trace_steady.py; the traces gzipped beside)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6w}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
tr() {
  rm -rf /tmp/t_$1
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/t_$1 -o t -- python3 $R/bench.py $2 --no-cpu-baseline --no-clock --steps 16 --warmup 4 > $O/b_$1.json 2> $O/b_$1.err || { echo "trace $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  f=$(find /tmp/t_$1 -name "*kernel_trace.csv" | head -1)
  gzip -c $f > $O/kt_$1.csv.gz
  python3 $R/tools/trace_steady.py $f > $O/steady_$1.json && python3 -c "
import json; d = json.load(open('$O/steady_$1.json')); b = json.loads([l for l in open('$O/b_$1.json') if l.startswith('{')][-1])
print('$1', round(b['value'] / 1e6, 2), {k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items() if k not in ('sum_ms', 'count')}, {k: round(v, 1) for k, v in d['sum_ms'].items()})"
}
tr hc "--workload c4h --components --inflight 2" && tr h "--workload c4h --inflight 2"
