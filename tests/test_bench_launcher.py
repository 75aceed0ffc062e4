"""bench.py's --gpus N launcher and the NUMA placement, on CPU (gloo, stub workload).

VERDICT r03 item 1: `python bench.py --gpus N` must start N ranks itself when no
launcher set WORLD_SIZE, relay exactly one JSON line with n_gpus = N, fail
loudly when a rank fails or WORLD_SIZE disagrees with --gpus, and bind every
rank's host threads to its GPU's NUMA node (sysfs, before HIP starts)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from corda_amd import numa  # noqa: E402


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(MASTER_ADDR="127.0.0.1", **kw)
    return env


def _bench(args, env, timeout=240):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_launcher_two_ranks_one_line():
    r = _bench(["--gpus", "2", "--workload", "stub", "--steps", "3", "--warmup", "1"], _env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1
    assert out["value"] > 0 and out["scaling"] == "weak"
    assert out["config"]["launcher"].startswith("torch.distributed.run (bench.py child)")
    assert len(out["config"]["numa_nodes_by_rank"]) == 2
    assert out["verdict_check"]["verdict_allgather_ok_all_ranks"] is True


def test_single_gpu_stays_in_process():
    r = _bench(["--gpus", "1", "--workload", "stub", "--steps", "2", "--warmup", "0"], _env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["config"]["launcher"] == "in-process"
    assert "verdict_allgather_ok_all_ranks" not in out["verdict_check"]


def test_failing_rank_fails_the_launch():
    r = _bench(["--gpus", "2", "--workload", "stub", "--steps", "1", "--warmup", "0"],
               _env(CORDA_BENCH_STUB_FAIL_RANK="1"))
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_world_size_must_match_gpus():
    r = _bench(["--gpus", "4", "--workload", "stub", "--steps", "1"],
               _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr


# ---- NUMA placement from a synthetic sysfs ---------------------------------------
def _fake_sysfs(tmp_path, gpus, cpu_nodes):
    """gpus: list of (simd_count, render_minor, location_id, numa_node); cpu_nodes: {node: cpulist}."""
    sysfs = tmp_path / "sys"
    base = sysfs / "class" / "kfd" / "kfd" / "topology" / "nodes"
    k = 0
    base.joinpath("0").mkdir(parents=True)
    base.joinpath("0", "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")  # the CPU node
    for simd, minor, loc, node in gpus:
        k += 1
        d = base / str(k)
        d.mkdir()
        d.joinpath("properties").write_text(
            "cpu_cores_count 0\nsimd_count %d\ndrm_render_minor %d\nlocation_id %d\ndomain 0\n" % (simd, minor, loc))
        r = sysfs / "class" / "drm" / ("renderD%d" % minor) / "device"
        r.mkdir(parents=True)
        r.joinpath("numa_node").write_text("%d\n" % node)
    for node, cl in cpu_nodes.items():
        n = sysfs / "devices" / "system" / "node" / ("node%d" % node)
        n.mkdir(parents=True)
        n.joinpath("cpulist").write_text(cl + "\n")
    return str(sysfs), str(tmp_path / "dev")  # no /dev/dri entries: every GPU counts as openable


def test_numa_map_and_visible_devices(tmp_path):
    sysfs, dev = _fake_sysfs(tmp_path, [(1024, 128, 0x0500, 0), (1024, 136, 0x1500, 0), (1024, 144, 0x8500, 1),
                                        (1024, 152, 0x9500, 1)], {0: "0-3", 1: "4-7"})
    env = {}
    assert [g["drm_render_minor"] for g in numa.gpu_nodes(sysfs, dev, env)] == [128, 136, 144, 152]
    assert numa.numa_of_gpu(2, sysfs, dev, env)["numa_node"] == 1
    assert numa.numa_of_gpu(4, sysfs, dev, env) is None
    env = {"HIP_VISIBLE_DEVICES": "3,0"}
    assert numa.numa_of_gpu(0, sysfs, dev, env)["drm_render_minor"] == 152
    assert numa.numa_of_gpu(1, sysfs, dev, env)["numa_node"] == 0
    env = {"ROCR_VISIBLE_DEVICES": "1,2,3", "CUDA_VISIBLE_DEVICES": "2"}
    assert numa.numa_of_gpu(0, sysfs, dev, env)["drm_render_minor"] == 152


def test_bind_rank_record(tmp_path):
    have = sorted(os.sched_getaffinity(0))
    cl = ",".join(str(c) for c in have[: max(1, len(have) // 2)])
    sysfs, dev = _fake_sysfs(tmp_path, [(1024, 128, 0x0500, 0), (1024, 136, 0x8500, 1)], {0: cl, 1: "100000"})
    rec = numa.bind_rank(0, sysfs, dev, env={}, apply=False)
    assert rec["numa_node"] == 0 and rec["cpus_bound"] == max(1, len(have) // 2)
    assert numa.location_matches(rec, 0x05, 0, 0) is True
    assert numa.location_matches(rec, 0x85, 0, 0) is False
    rec = numa.bind_rank(1, sysfs, dev, env={}, apply=False)  # node 1's CPUs are not ours: no binding
    assert rec["numa_node"] == 1 and rec["cpus_bound"] is None and "affinity" in rec["numa_reason"]
    rec = numa.bind_rank(5, sysfs, dev, env={}, apply=False)
    assert rec["numa_node"] is None


def test_parse_cpulist():
    assert numa.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert numa.parse_cpulist("") == []
