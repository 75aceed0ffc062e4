"""Host-side NUMA placement for one-process-per-GPU ranks.

Each bench rank (and any JVM-side worker that owns one GPU) should run its
host threads -- the C oracle checks, the CSR packing pool of
`cordahip_sig_verify`, the pinned-buffer first touch -- on the NUMA node its
GPU hangs off, so pinned staging sits next to the PCIe root port that DMAs it.
The mapping is read from sysfs WITHOUT touching the GPU runtime (it must be
decided before HIP starts its threads, which inherit the affinity):

  HIP device i = the i-th GPU node of the KFD topology (nodes with
  simd_count > 0, in node order) whose render node the process may open,
  after ROCR_VISIBLE_DEVICES and then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES
  select from that list -- the order ROCr enumerates agents and HIP devices.
  Its NUMA node is /sys/class/drm/renderD<minor>/device/numa_node, its CPUs
  /sys/devices/system/node/node<N>/cpulist (intersected with the current
  affinity, so a cgroup's CPU set is respected).

`bind_rank` returns a record for the bench line; after HIP is up the caller
can confirm the choice by comparing the PCI location with the device's
properties (`location_matches`).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def parse_cpulist(s: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]"""
    out: List[int] = []
    for part in s.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _props(text: str) -> Dict[str, int]:
    d: Dict[str, int] = {}
    for line in text.splitlines():
        kv = line.split()
        if len(kv) == 2:
            try:
                d[kv[0]] = int(kv[1])
            except ValueError:
                pass
    return d


def _select(items: list, spec: Optional[str]) -> list:
    """Apply a *_VISIBLE_DEVICES list of integer indices (UUID forms are not handled: keep all)."""
    if spec is None or spec.strip() == "":
        return items
    try:
        idx = [int(x) for x in spec.split(",") if x.strip() != ""]
    except ValueError:
        return items
    return [items[i] for i in idx if 0 <= i < len(items)]


def gpu_nodes(sysfs: str = "/sys", dev: str = "/dev", env=None) -> List[Dict[str, int]]:
    """KFD GPU nodes in HIP device order (see module docstring)."""
    env = os.environ if env is None else env
    base = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        names = sorted((n for n in os.listdir(base) if n.isdigit()), key=int)
    except OSError:
        return []
    gpus = []
    for n in names:
        p = _props(_read(os.path.join(base, n, "properties")) or "")
        if p.get("simd_count", 0) <= 0:
            continue  # a CPU node
        minor = p.get("drm_render_minor")
        if minor is None:
            continue
        rnode = os.path.join(dev, "dri", "renderD%d" % minor)
        if os.path.exists(rnode) and not os.access(rnode, os.R_OK | os.W_OK):
            continue  # ROCr skips GPUs it cannot open
        p["kfd_node"] = int(n)
        gpus.append(p)
    gpus = _select(gpus, env.get("ROCR_VISIBLE_DEVICES"))
    gpus = _select(gpus, env.get("HIP_VISIBLE_DEVICES") or env.get("CUDA_VISIBLE_DEVICES"))
    return gpus


def numa_of_gpu(local_rank: int, sysfs: str = "/sys", dev: str = "/dev", env=None) -> Optional[Dict[str, int]]:
    gpus = gpu_nodes(sysfs, dev, env)
    if not 0 <= local_rank < len(gpus):
        return None
    g = gpus[local_rank]
    raw = _read(os.path.join(sysfs, "class", "drm", "renderD%d" % g["drm_render_minor"], "device", "numa_node"))
    try:
        node = int(raw.strip()) if raw is not None else -1
    except ValueError:
        node = -1
    return {"numa_node": node, "location_id": g.get("location_id", -1), "domain": g.get("domain", 0),
            "drm_render_minor": g["drm_render_minor"], "kfd_node": g["kfd_node"]}


def node_cpus(node: int, sysfs: str = "/sys") -> List[int]:
    raw = _read(os.path.join(sysfs, "devices", "system", "node", "node%d" % node, "cpulist"))
    return parse_cpulist(raw) if raw else []


def bind_rank(local_rank: int, sysfs: str = "/sys", dev: str = "/dev", env=None, apply: bool = True) -> Dict:
    """Pin this process (and the threads it creates later) to its GPU's NUMA node.

    Returns a record for the bench line: numa_node (or None), the number of CPUs
    bound, and why nothing was bound when that is the case."""
    rec: Dict = {"numa_node": None, "cpus_bound": None}
    info = numa_of_gpu(local_rank, sysfs, dev, env)
    if info is None:
        rec["numa_reason"] = "no KFD topology entry for local rank %d" % local_rank
        return rec
    rec.update({"numa_node": info["numa_node"], "gpu_location_id": info["location_id"],
                "gpu_pci_domain": info["domain"]})
    if info["numa_node"] < 0:
        rec["numa_reason"] = "GPU reports no NUMA node"
        return rec
    have = sorted(os.sched_getaffinity(0))
    want = sorted(set(node_cpus(info["numa_node"], sysfs)) & set(have))
    if not want:
        rec["numa_reason"] = "no CPU of node %d in this process's affinity" % info["numa_node"]
        return rec
    if apply:
        os.sched_setaffinity(0, want)
    rec["cpus_bound"] = len(want)
    return rec


def location_matches(rec: Dict, pci_bus: int, pci_device: int, pci_domain: int = 0) -> Optional[bool]:
    """Compare the KFD location_id chosen before HIP init (bus << 8 | device << 3 | function)
    with the PCI address HIP reports for the device the rank actually opened."""
    loc = rec.get("gpu_location_id")
    if loc is None or loc < 0:
        return None
    return (loc >> 8) == pci_bus and ((loc >> 3) & 0x1F) == pci_device and rec.get("gpu_pci_domain", 0) == pci_domain
