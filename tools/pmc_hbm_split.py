"""Apply the Ed25519 ladder's Infinity-Cache (MALL) split to a composed PMC
profile (tools/pmc_compose.py output): the ladder's measured FETCH_SIZE bytes are
L2-to-fabric bytes, MALL hits included; tools/mall_sim.cpp (calibrated on the
measured ladder fetch of C2, profiles/r04_pmc_ed25519_split.json) puts 0.369 of
them in HBM. Every other kernel's bytes (prep's streaming record writes, the
ids' leaf reads, the ECDSA kernels) stay as counted: an upper bound on HBM.

usage: pmc_hbm_split.py composed.json > split.json"""
import json
import sys

HBM_FRACTION = 0.369  # profiles/r04_mall_model.jsonl: mean of the lockstep and staggered schedules


def main():
    d = json.load(open(sys.argv[1]))
    lanes = d["lanes_per_pass"]
    lad = [v for k, v in d["kernels"].items() if "ed25519_ladder" in k and v.get("in_total", True)]
    fetch = sum(v["counters"].get("FETCH_SIZE", 0.0) * 1024 * 2 for v in lad) / lanes  # KB, x2 gfx950 correction
    total = d["hbm_bytes_per_unit"]
    mall = fetch * (1 - HBM_FRACTION)
    d["l2_fabric_bytes_per_unit"] = total
    d["mall_bytes_per_unit"] = mall
    d["hbm_bytes_per_unit"] = total - mall
    d["hbm_split"] = {
        "method": "the Ed25519 ladder's measured fetch split by tools/mall_sim.cpp's HBM fraction (%.3f, calibrated on "
                  "C2's ladder, profiles/r04_pmc_ed25519_split.json); every other kernel's FETCH/WRITE bytes counted "
                  "as HBM (an upper bound: their MALL hits are not modelled)" % HBM_FRACTION,
        "ladder_fetch_bytes_per_unit": fetch, "ladder_mall_bytes_per_unit": mall,
        "hbm_over_algorithmic": (total - mall) / d["algorithmic_bytes_per_unit"],
        "fabric_over_algorithmic": total / d["algorithmic_bytes_per_unit"]}
    json.dump(d, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
