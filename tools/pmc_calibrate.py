"""Check the VALU counters' units against the VALU issue-cost microbenchmark.

Input: the stdout of tools/microbench/valu_rates.hip (one JSON line per op:
measured cycles per wave64 instruction at 8 waves/SIMD, i.e. a kernel that is
VALU-issue bound by construction) and tools/pmc_summary.py's per-kernel sums
of a rocprofv3 --pmc pass over the same binary. For each op kernel: the
counter ratio SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU next to the measured
cycles per instruction, and SQ_ACTIVE_INST_VALU over the SIMD-cycles the
kernel had (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), which must be ~1 for these
kernels if the counter measures VALU issue cycles.

usage: pmc_calibrate.py valu_rates.jsonl summary.json > calibration.json
"""
import json
import re
import sys


def main():
    rates = [json.loads(l) for l in open(sys.argv[1]) if l.strip().startswith("{")]
    ops = [r for r in rates if "op" in r]
    summ = json.load(open(sys.argv[2]))
    # kernels are bench<K> templates in enum order, K = 0..N-1
    by_k = {}
    for name, c in summ.items():
        m = re.search(r"bench<(\d+)>", name)
        if m:
            by_k[int(m.group(1))] = c
    rows = []
    for k, r in enumerate(ops):
        c = by_k.get(k)
        if not c:
            continue
        row = {"op": r["op"], "measured_cycles_per_wave_inst": r["cycles_per_wave_inst"]}
        if c.get("SQ_INSTS_VALU"):
            row["active_inst_valu_per_inst"] = c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_INSTS_VALU"]
        if c.get("GRBM_GUI_ACTIVE"):
            simd_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 1024
            row["active_inst_valu_over_simd_cycles"] = c.get("SQ_ACTIVE_INST_VALU", 0) / simd_cycles
            row["insts_x_measured_over_simd_cycles"] = c.get("SQ_INSTS_VALU", 0) * r["cycles_per_wave_inst"] / simd_cycles
        if c.get("SQ_BUSY_CYCLES"):
            row["active_inst_valu_over_busy_cycles"] = c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_BUSY_CYCLES"]
        row["counters"] = c
        rows.append(row)
    print(json.dumps({"source": "tools/microbench/valu_rates.hip under rocprofv3 --pmc", "ops": rows}, indent=1))


if __name__ == "__main__":
    main()
