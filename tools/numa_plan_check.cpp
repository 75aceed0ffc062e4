// The library's NUMA placement rule (corda_amd/csrc/numa_place.hpp) on a given
// sysfs tree: tests/test_numa_plan.py drives it from a fake tree (2 nodes, 8
// GPUs) and checks the plan; on a real box it prints the plan the library's
// contexts would use.
//
// usage: numa_plan_check SYSFS_ROOT ALLOWED_CPULIST CAP PCI [PCI ...]
// prints one JSON line: {"devices": [{"pci", "node", "cpus", "threads", "why"}, ...]}
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../corda_amd/csrc/numa_place.hpp"

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: numa_plan_check SYSFS_ROOT ALLOWED_CPULIST CAP PCI [PCI ...]\n");
    return 2;
  }
  const std::vector<int> allowed = cordahip::rt::parse_cpulist(argv[2]);
  std::vector<std::string> pci(argv + 4, argv + argc);
  const auto plan = cordahip::rt::numa_plan(argv[1], pci, allowed, atoi(argv[3]));
  printf("{\"devices\": [");
  for (size_t i = 0; i < plan.size(); i++) {
    printf("%s{\"pci\": \"%s\", \"node\": %d, \"threads\": %d, \"why\": \"%s\", \"cpus\": [", i ? ", " : "",
           pci[i].c_str(), plan[i].node, plan[i].threads, plan[i].why.c_str());
    for (size_t k = 0; k < plan[i].cpus.size(); k++) printf("%s%d", k ? ", " : "", plan[i].cpus[k]);
    printf("]}");
  }
  printf("]}\n");
  return 0;
}
