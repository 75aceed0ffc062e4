# r06: NUMA placement on the box -- the plan the library uses, pack_bench with one bound pool per
# simulated device, host-batch tests, c2h / c3h / c4h with the per-device pools
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6k
mkdir -p $O
cd $R
g++ -O2 -std=c++17 -pthread -o /tmp/pack_bench tools/pack_bench.cpp && g++ -O2 -std=c++17 -o /tmp/npc tools/numa_plan_check.cpp || exit 1
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpus', os.cpu_count())"
ls /sys/devices/system/node/ | grep node | tr '\n' ' '; echo
PCI=$(python3 -c "
import torch; p = torch.cuda.get_device_properties(0)
print('%04x:%02x:%02x.0' % (getattr(p, 'pci_domain_id', 0), p.pci_bus_id, p.pci_device_id))")
echo "gpu pci $PCI"
/tmp/npc /sys "$(python3 -c "import os; print(','.join(map(str, sorted(os.sched_getaffinity(0)))))")" 16 $PCI | tee $O/numa_plan_box.json
timeout -k 10 120 /tmp/pack_bench $((1<<22)) 16 8 | tee $O/pack_pools8.jsonl
timeout -k 10 120 /tmp/pack_bench $((1<<22)) 16 1 | tee $O/pack_pools1.jsonl
timeout -k 10 120 /tmp/pack_bench $((1<<22)) 16 2 | tee $O/pack_pools2.jsonl
CORDAHIP_TRACE=1 timeout -k 10 120 python -c "
from corda_amd.engine import Engine
with Engine(1) as e: print('devices', e.device_count)" 2>&1 | grep -i "numa\|devices" | tee $O/trace_init.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_batch.py tests/test_gpu_runtime.py tests/test_gpu_multidevice.py tests/test_gpu_csr.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-clock --steps 5 --warmup 1 $2 > $O/b_$1.json 2> $O/b_$1.err || { echo "bench $1 failed"; tail -20 $O/b_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: v for k, v in d['verdict_check'].items() if 'mismatch' in k})"
}
run c2h "--workload c2h" && run c3h "--workload c3h" && run c4h2 "--workload c4h --inflight 2"
