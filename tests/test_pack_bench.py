"""The host budget of one process feeding several GPUs:
tools/pack_bench.cpp runs the generic batch's per-lane host work -- classify,
pack the row, scatter the status back, build the verdict words -- with the
library's own code (corda_amd/csrc/pack_rows.hpp) on the CPU, single- and
multi-threaded, for Ed25519 and ECDSA batches. DESIGN §7 turns its lanes/s per
thread into the threads 8 GPUs at 1.1e8 verifications/s each would need."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pack_bench_runs_and_scales(tmp_path):
    exe = str(tmp_path / "pack_bench")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-o", exe,
                           os.path.join(ROOT, "tools", "pack_bench.cpp")])
    threads = max(1, min(4, os.cpu_count() or 1))
    out = subprocess.run([exe, str(1 << 20), str(threads)], capture_output=True, text=True, check=True, timeout=120)
    rows = [json.loads(x) for x in out.stdout.splitlines()]
    by = {(r["scheme"], r["threads"]): r for r in rows}
    assert ("ed25519", 1) in by and ("ecdsa", 1) in by
    for r in rows:
        assert r["lanes"] == 1 << 20 and r["lanes_per_s"] > 1e6
    # packing is memcpy-bound: a thread packs millions of lanes per second, far more
    # than one GPU verifies per thread of the GPU's host
    assert by[("ed25519", 1)]["lanes_per_s"] > 5e6 and by[("ecdsa", 1)]["lanes_per_s"] > 3e6


def test_pack_bench_pools_mode(tmp_path):
    """one bound pool per simulated device (the library's per-device NUMA pools):
    every pool packs its own shard at once; the aggregate is reported"""
    exe = str(tmp_path / "pack_bench")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-o", exe,
                           os.path.join(ROOT, "tools", "pack_bench.cpp")])
    pools = 2
    out = subprocess.run([exe, str(1 << 18), str(2 * pools), str(pools)], capture_output=True, text=True, check=True,
                         timeout=120)
    rows = [json.loads(x) for x in out.stdout.splitlines()]
    assert {r["scheme"] for r in rows} == {"ed25519", "ecdsa"}
    for r in rows:
        assert r["pools"] == pools and r["threads_per_pool"] == 2 and r["lanes_per_s"] > 1e6
