"""The library's per-device NUMA placement (corda_amd/csrc/numa_place.hpp, used by
cordahip_init for every context device: a host pool bound to CPUs of the GPU's
node, the pipeline threads bound there while they pack and first-touch pinned
stages) driven from a fake sysfs tree through tools/numa_plan_check.cpp, which
compiles the same header: 2 NUMA nodes x 48 CPUs, 8 GPUs (4 per node), a cgroup
that allows only part of the machine, GPUs with no node, more GPUs than CPUs."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ absent")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("numa") / "numa_plan_check")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-fsanitize=address,undefined", "-o", out,
                           os.path.join(ROOT, "tools", "numa_plan_check.cpp")])
    return out


GPUS = ["0000:%02x:00.0" % b for b in (0x05, 0x15, 0x25, 0x35, 0x85, 0x95, 0xa5, 0xb5)]


def fake_sysfs(root, nodes, gpu_node):
    for n, cpus in nodes.items():
        d = root / "devices" / "system" / "node" / ("node%d" % n)
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus + "\n")
    for pci, n in gpu_node.items():
        d = root / "bus" / "pci" / "devices" / pci
        d.mkdir(parents=True)
        (d / "numa_node").write_text("%d\n" % n)
    return str(root)


def plan(exe, root, allowed, cap, pcis):
    out = subprocess.check_output([exe, root, allowed, str(cap)] + pcis, text=True)
    return json.loads(out)["devices"]


def test_two_nodes_eight_gpus(exe, tmp_path):
    root = fake_sysfs(tmp_path, {0: "0-47", 1: "48-95"}, {g: (0 if i < 4 else 1) for i, g in enumerate(GPUS)})
    p = plan(exe, root, "0-95", 16, GPUS)
    assert [d["node"] for d in p] == [0, 0, 0, 0, 1, 1, 1, 1]
    # each node's 48 CPUs split into disjoint slices of 12, one per GPU, in device order
    assert [d["cpus"] for d in p[:4]] == [list(range(12 * k, 12 * k + 12)) for k in range(4)]
    assert [d["cpus"] for d in p[4:]] == [list(range(48 + 12 * k, 60 + 12 * k)) for k in range(4)]
    assert all(d["threads"] == 12 for d in p)
    # the per-device cap
    assert all(d["threads"] == 8 for d in plan(exe, root, "0-95", 8, GPUS))


def test_cgroup_and_unknown_nodes(exe, tmp_path):
    gmap = {g: (0 if i < 4 else 1) for i, g in enumerate(GPUS)}
    gmap[GPUS[7]] = -1  # no NUMA node reported
    root = fake_sysfs(tmp_path, {0: "0-47", 1: "48-95"}, gmap)
    # the process may use 16 CPUs: 8 on each node
    p = plan(exe, root, "40-55", 16, GPUS + ["0000:ff:00.0"])
    assert [d["cpus"] for d in p[:4]] == [[40, 41], [42, 43], [44, 45], [46, 47]]
    assert [d["cpus"] for d in p[4:7]] == [[48, 49], [50, 51, 52], [53, 54, 55]]
    assert p[7]["cpus"] == [] and p[7]["node"] == -1 and "no NUMA node" in p[7]["why"]
    assert p[8]["cpus"] == [] and "no sysfs" in p[8]["why"]  # a PCI address sysfs does not know
    assert p[7]["threads"] == 16 and p[0]["threads"] == 2  # unbound: the whole allowed set


def test_more_gpus_than_cpus_and_no_cpus_on_node(exe, tmp_path):
    root = fake_sysfs(tmp_path, {0: "0-1", 1: "2-3"}, {g: (0 if i < 4 else 1) for i, g in enumerate(GPUS)})
    p = plan(exe, root, "0-1", 16, GPUS)
    assert all(d["cpus"] in ([0], [1], [0, 1]) for d in p[:4]) and all(d["threads"] >= 1 for d in p)
    assert all(d["cpus"] == [] and "affinity" in d["why"] for d in p[4:])  # node 1's CPUs not allowed
