"""Compose the committed PMC profile (profiles/rNN_pmc_*.json) from the passes of
tools/gpu_pmc.sh (summed per kernel by tools/pmc_summary.py).

Per kernel and in total: VALU instructions per lane (SQ_INSTS_VALU counts
wave64 instructions; x64 / lanes = lane-instructions per lane), VALU issue cycles per
wave-instruction (SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU), VALU-busy fraction
measured directly (SQ_ACTIVE_INST_VALU over the SIMD-cycles the kernel had:
GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) and, for comparison, the round-1
estimate (4 cycles per wave-instruction); HBM bytes per lane from FETCH_SIZE
(doubled, the gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md) and
WRITE_SIZE (as read), each from its own pass. The counters' units are checked
against tools/microbench/valu_rates.hip (tools/pmc_calibrate.py).

Corpus-generation and one-time table kernels (signers, fixed-base tables) are
listed but left out of the total: the total is the verification pipeline.

usage: pmc_compose.py summary.json LANES "command" ALG_BYTES_PER_UNIT "note" > out.json
"""
import json
import sys

SIMDS = 1024
XCDS = 8
NOT_TIMED = ("sign_kernel", "gtable_kernel", "btable_kernel")


def derive(c, lanes):
    d = {}
    insts = c.get("SQ_INSTS_VALU")
    active = c.get("SQ_ACTIVE_INST_VALU")
    gui = c.get("GRBM_GUI_ACTIVE")
    if insts:
        d["valu_wave_insts_per_lane"] = insts / lanes
        d["valu_lane_insts_per_lane"] = insts * 64 / lanes
    if insts and active:
        d["valu_issue_cycles_per_wave_inst"] = active / insts
    if gui:
        simd_cycles = gui / XCDS * SIMDS
        if active:
            d["valu_busy_direct"] = active / simd_cycles
        if insts:
            d["valu_busy_est_4cyc"] = insts * 4 / simd_cycles
    if "FETCH_SIZE" in c:  # KB
        d["hbm_fetch_bytes_per_lane"] = c["FETCH_SIZE"] * 1024 * 2 / lanes
    if "WRITE_SIZE" in c:
        d["hbm_write_bytes_per_lane"] = c["WRITE_SIZE"] * 1024 / lanes
    return d


def main():
    summ, lanes, cmd, alg, note = sys.argv[1], float(sys.argv[2]), sys.argv[3], float(sys.argv[4]), sys.argv[5]
    s = json.load(open(summ))
    kernels = {}
    tot = {}
    for k, c in s.items():
        kernels[k] = {"counters": c, "derived": derive(c, lanes)}
        if any(t in k for t in NOT_TIMED):
            kernels[k]["in_total"] = False
            continue
        for n, v in c.items():
            if n != "dispatches_per_pass":
                tot[n] = tot.get(n, 0.0) + v
    td = derive(tot, lanes)
    out = {
        "command": cmd,
        "lanes_per_pass": int(lanes),
        "kernels": kernels,
        "total": {"counters": tot, "derived": td},
        "hbm_bytes_per_unit": td.get("hbm_fetch_bytes_per_lane", 0) + td.get("hbm_write_bytes_per_lane", 0),
        "algorithmic_bytes_per_unit": alg,
        "note": note,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
