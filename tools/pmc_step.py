"""Compose one bench step's PMC profile (profiles/r06_pmc_<workload>.json) from
counter passes of two runs of the same bench command: --steps 1 and --steps 2
(--warmup 0 --no-clock --no-cpu-baseline). Their difference is exactly the
second timed step's kernels -- corpus generation, the init step, the checks and
the first call's one-time work (shape builds, workspace growth) cancel -- so
every line's roofline fields come from a PMC of its own workload.

Counters (tools/gpu_pmc_step.sh): pass A = SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE, pass B = FETCH_SIZE, pass C = WRITE_SIZE,
each in its own run. Derived as tools/pmc_compose.py does (FETCH_SIZE x2, the
gfx950 correction; VALU busy from SQ_INSTS_VALU x 4 cycles and directly from
SQ_ACTIVE_INST_VALU over GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), per unit of the
bench line (signatures per step, from the steps-2 run's JSON line). Ed25519
workloads also get the ladder's Infinity-Cache split (tools/pmc_hbm_split.py's
calibrated HBM fraction) as traffic_hbm_modeled; the counters stay primary
(l2_fabric_bytes_per_unit).

usage: pmc_step.py DIR WORKLOAD_TAG "bench args" ALG_BYTES_PER_UNIT > out.json
  DIR holds s1_A.csv s1_B.csv s1_C.csv s2_A.csv s2_B.csv s2_C.csv and s2_line.json (dev tool)
"""
import csv
import json
import os
import sys
from collections import defaultdict

SIMDS, XCDS = 1024, 8
HBM_FRACTION = 0.369  # tools/pmc_hbm_split.py (the ladder's MALL model, calibrated on C2)
ONE_TIME = ("sign_kernel", "gtable_kernel", "btable_kernel")


def sums(path):
    out = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if "cordahip" not in k:
            continue
        out[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return out, {k: len(v) for k, v in disp.items()}


def derive(c, units):
    d = {}
    insts, active, gui = c.get("SQ_INSTS_VALU"), c.get("SQ_ACTIVE_INST_VALU"), c.get("GRBM_GUI_ACTIVE")
    if insts:
        d["valu_wave_insts_per_lane"] = insts / units
        d["valu_lane_insts_per_lane"] = insts * 64 / units
    if insts and active:
        d["valu_issue_cycles_per_wave_inst"] = active / insts
    if gui:
        simd_cycles = gui / XCDS * SIMDS
        if active:
            d["valu_busy_direct"] = active / simd_cycles
        if insts:
            d["valu_busy_est_4cyc"] = insts * 4 / simd_cycles
    if "FETCH_SIZE" in c:
        d["hbm_fetch_bytes_per_lane"] = c["FETCH_SIZE"] * 1024 * 2 / units
    if "WRITE_SIZE" in c:
        d["hbm_write_bytes_per_lane"] = c["WRITE_SIZE"] * 1024 / units
    return d


def main():
    dr, tag, cmd, alg = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4])
    line = json.load(open(os.path.join(dr, "s2_line.json")))
    units = line["value"] * line["ms_per_step"] / 1e3 / line["n_gpus"]  # units per step per GPU
    kern = defaultdict(dict)
    disp = {}
    for g in "ABC":
        a, da = sums(os.path.join(dr, "s1_%s.csv" % g))
        b, db = sums(os.path.join(dr, "s2_%s.csv" % g))
        for k in set(a) | set(b):
            for n in set(a.get(k, {})) | set(b.get(k, {})):
                kern[k][n] = b.get(k, {}).get(n, 0.0) - a.get(k, {}).get(n, 0.0)
            disp[k] = db.get(k, 0) - da.get(k, 0)
    kernels, tot = {}, defaultdict(float)
    for k, c in sorted(kern.items()):
        if disp.get(k, 0) <= 0 or any(t in k for t in ONE_TIME):
            continue  # not a kernel of the timed step
        kernels[k] = {"counters": dict(c), "dispatches_per_step": disp[k], "derived": derive(c, units)}
        for n, v in c.items():
            tot[n] += v
    td = derive(tot, units)
    fabric = td.get("hbm_fetch_bytes_per_lane", 0) + td.get("hbm_write_bytes_per_lane", 0)
    out = {"command": "tools/gpu_pmc_step.sh: rocprofv3 --pmc, 3 passes x (--steps 1, --steps 2) of "
                      "bench.py %s --warmup 0 --no-clock --no-cpu-baseline; one step = the difference" % cmd,
           "workload": tag, "units_per_step": units, "lanes_per_pass": int(round(units)),
           "kernels": kernels, "total": {"counters": dict(tot), "derived": td},
           "l2_fabric_bytes_per_unit": fabric, "hbm_bytes_per_unit": fabric, "algorithmic_bytes_per_unit": alg,
           "note": "L2-to-fabric bytes (FETCH_SIZE x2 + WRITE_SIZE) of the kernels of one timed step per unit; "
                   "Infinity-Cache hits included"}
    lad = [v for k, v in kernels.items() if "ed25519_ladder" in k]
    if lad:
        lf = sum(v["counters"].get("FETCH_SIZE", 0.0) * 1024 * 2 for v in lad) / units
        mall = lf * (1 - HBM_FRACTION)
        out["mall_bytes_per_unit"] = mall
        out["hbm_bytes_per_unit"] = fabric - mall
        out["hbm_split"] = {"method": "the Ed25519 ladder's measured fetch split by tools/mall_sim.cpp's HBM fraction "
                                      "(%.3f); every other kernel's bytes counted as HBM (an upper bound)" % HBM_FRACTION,
                            "ladder_fetch_bytes_per_unit": lf, "ladder_mall_bytes_per_unit": mall}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
