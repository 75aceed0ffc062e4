"""Radix 2^32 vs radix 2^29 field-product A/B -> profiles/r05_radix32_ab.json.

Builds and runs tools/microbench/p256_radix32 (hipcc, here on the GPU box),
checks the radix-32 P-256 product / square and GF(2^255-19) product of 512
random lanes against Python integers, and records the time per field op of
every variant next to the VALU instructions of its loop body (hipcc -S of the
same source, tools/isa_blocks.py: 4 products per loop body). Adoption rule:
radix 2^32 only at >= 10% less time per product than the production radix-2^29
asm product; otherwise this file is the committed negative result and DESIGN
§8b says so."""
import json
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SRC = os.path.join(HERE, "p256_radix32.hip")
P256 = 2**256 - 2**224 + 2**192 + 2**96 - 1
P25519 = 2**255 - 19
KINDS = ["r29_mul_p256_asm", "r29_sqr_p256_asm", "p32_mul_p256_nist", "p32_sqr_p256_nist", "q32_mul_25519",
         "fe_mul_25519_radix25.5"]


def isa_counts():
    s = "/tmp/p256_radix32.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                           "-S", "-o", s, SRC], stderr=subprocess.DEVNULL)
    out = {}
    for k, name in enumerate(KINDS):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_blocks.py"), s, "chainILi%dE" % k, "100"],
                           capture_output=True, text=True, check=True)
        best = max(r.stdout.splitlines(), key=lambda ln: int(re.search(r"VALU\s+(\d+)", ln).group(1)))
        valu = int(re.search(r"VALU\s+(\d+)", best).group(1))
        total = int(re.search(r"total\s+(\d+)", best).group(1))
        nops = int(m.group(1)) if (m := re.search(r"s_nop (\d+)", best)) else 0
        out[name] = {"valu_per_op": valu / 4, "instructions_per_op": total / 4, "s_nop_per_op": nops / 4,
                     "loop_body_mix": best.split("|")[1].strip()}
    return out


def main():
    exe = "/tmp/p256_radix32"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-o", exe, SRC],
                          stderr=subprocess.DEVNULL)
    r = subprocess.run([exe] + sys.argv[1:2], capture_output=True, text=True, check=True, timeout=300)
    bench, bad, n = [], [], 0
    val = lambda w: sum(x << (32 * k) for k, x in enumerate(w))  # noqa: E731
    for ln in r.stdout.splitlines():
        if ln.startswith("{"):
            bench.append(json.loads(ln))
        elif ln.startswith("CHK"):
            v = [int(x) for x in ln.split()[1:]]
            A, B, m, s, q = val(v[0:8]), val(v[8:16]), val(v[16:24]), val(v[24:32]), val(v[32:40])
            ok = ((m - A * B) % P256 == 0 and m < 2 * P256 and (s - A * A) % P256 == 0 and s < 2 * P256
                  and (q - A * B) % P25519 == 0)
            if not ok:
                bad.append(n)
            n += 1
    t = {x["bench"]: x["ps_per_field_op"] for x in bench}
    isa = isa_counts()
    ratio = {"p256_mul": t["p32_mul_p256_nist"] / t["r29_mul_p256_asm"],
             "p256_sqr": t["p32_sqr_p256_nist"] / t["r29_sqr_p256_asm"],
             "25519_mul": t["q32_mul_25519"] / t["fe_mul_25519_radix25.5"]}
    res = {
        "what": "radix 2^32 x 8 (v_mad_u64_u32 + v_addc_co_u32 per MAC, 3-word column accumulator; P-256: NIST "
                "word-aligned reduction; 2^255-19: fold x38) against the production radix-2^29 special-form "
                "Montgomery asm products (fp29_asm.hpp f29a_mul_r1 / f29a_sqr_r1) and the radix-2^25.5 fe_mul, "
                "same harness (4 independent chains per lane, 2^20 lanes, 2 waves/SIMD), one MI355X",
        "bench": bench,
        "exactness": {"lanes_checked": n, "mismatches": len(bad), "first_bad": bad[:5],
                      "rule": "p32 mul / sqr == A*B, A^2 mod p and < 2p; q32 mul == A*B mod 2^255-19 "
                              "(Python integers)"},
        "isa_per_op": isa,
        "time_ratio_radix32_over_production": ratio,
        "adopt_threshold": "radix-32 product >= 10% faster (ratio <= 0.90)",
    }
    res["adopted"] = ratio["p256_mul"] <= 0.90 and not bad
    res["verdict"] = ("adopted" if res["adopted"] else
                      "not adopted: every radix-2^32 MAC needs the carry out of bit 64 counted (v_addc_co_u32 on "
                      "VCC, plus s_nop for the VCC hazard) and every column end moves the 3-word accumulator down, "
                      "so the 64-MAC product alone exceeds the radix-2^29 product with its special-form REDC, "
                      "before the word-aligned reduction's signed carry passes")
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "r05_radix32_ab.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("exactness", "time_ratio_radix32_over_production", "adopted")}))
    print(json.dumps({k: v["valu_per_op"] for k, v in isa.items()}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
