// NUMA placement of a context's per-device host work (packing, scattering,
// reduce; the pinned staging those threads first-touch): each device gets a
// pool of host threads bound to CPUs of the NUMA node its GPU hangs off, so the
// rows it packs and the pinned stages PCIe reads from sit next to that GPU's
// root port. One JVM context drives every GPU of the node (the
// shards are independent, SignedTransaction.kt:97-99); corda_amd/numa.py does the
// same per process for one-rank-per-GPU launches.
//
// The rule (sysfs only, no HIP here, so tools/numa_plan_check.cpp runs it on a
// fake tree): device i's node = /sys/bus/pci/devices/<its PCI address>/numa_node
// (-1 or absent: no node); a node's CPUs = /sys/devices/system/node/node<N>/cpulist
// intersected with the CPUs the process may use. The devices of one node split
// its CPUs into disjoint, contiguous slices (in device order); a device whose
// node is unknown, or whose slice would be empty, takes the whole allowed set
// unbound (no pinning). threads = min(slice size, per_device cap).
#pragma once
#include <algorithm>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

namespace cordahip {
namespace rt {

inline std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    const std::string part = s.substr(i, j - i);
    const size_t dash = part.find('-');
    char* end = nullptr;
    if (!part.empty() && part.find_first_not_of(" \n\t") != std::string::npos) {
      if (dash == std::string::npos) {
        const long v = strtol(part.c_str(), &end, 10);
        if (end != part.c_str()) out.push_back((int)v);
      } else {
        const long a = strtol(part.substr(0, dash).c_str(), nullptr, 10);
        const long b = strtol(part.substr(dash + 1).c_str(), nullptr, 10);
        for (long v = a; v <= b && v - a < 65536; v++) out.push_back((int)v);
      }
    }
    i = j + 1;
  }
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return out;
}

inline bool read_text(const std::string& path, std::string& out) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096];
  out.clear();
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, k);
  fclose(f);
  return true;
}

struct NumaPlace {
  int node = -1;          // the GPU's NUMA node (-1: unknown)
  std::vector<int> cpus;  // the device pool's CPUs (empty: unbound)
  int threads = 1;
  std::string why;        // why nothing was bound, when that is the case
};

// pci[i]: device i's PCI address ("0000:0c:00.0"); allowed: the process's CPUs;
// cap: threads per device at most (CORDAHIP_HOST_THREADS, default 16)
inline std::vector<NumaPlace> numa_plan(const std::string& sysfs, const std::vector<std::string>& pci,
                                        const std::vector<int>& allowed, int cap) {
  std::vector<NumaPlace> out(pci.size());
  std::map<int, std::vector<size_t>> by_node;
  for (size_t i = 0; i < pci.size(); i++) {
    std::string t;
    if (pci[i].empty() || !read_text(sysfs + "/bus/pci/devices/" + pci[i] + "/numa_node", t)) {
      out[i].why = "no sysfs numa_node for the GPU";
      continue;
    }
    out[i].node = (int)strtol(t.c_str(), nullptr, 10);
    if (out[i].node < 0) {
      out[i].why = "the GPU reports no NUMA node";
      continue;
    }
    by_node[out[i].node].push_back(i);
  }
  for (auto& kv : by_node) {
    std::string t;
    std::vector<int> cpus;
    if (read_text(sysfs + "/devices/system/node/node" + std::to_string(kv.first) + "/cpulist", t)) cpus = parse_cpulist(t);
    std::vector<int> mine;
    std::set_intersection(cpus.begin(), cpus.end(), allowed.begin(), allowed.end(), std::back_inserter(mine));
    const size_t nd = kv.second.size();
    for (size_t k = 0; k < nd; k++) {
      NumaPlace& p = out[kv.second[k]];
      const size_t lo = mine.size() * k / nd, hi = mine.size() * (k + 1) / nd;
      if (hi > lo) {
        p.cpus.assign(mine.begin() + (long)lo, mine.begin() + (long)hi);
      } else if (!mine.empty()) {  // more devices than CPUs on the node: share them all
        p.cpus = mine;
      } else {
        p.why = "no CPU of the GPU's node in this process's affinity";
      }
    }
  }
  for (NumaPlace& p : out) {
    const int avail = p.cpus.empty() ? (int)allowed.size() : (int)p.cpus.size();
    p.threads = std::max(1, std::min(cap, avail));
  }
  return out;
}

}  // namespace rt
}  // namespace cordahip
