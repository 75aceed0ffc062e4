#!/usr/bin/env python3
"""Writes corda_amd/csrc/fp29_consts.hpp: the constants of fp29.hpp's radix-2^29
Montgomery representation (R = 2^261) of the secp256k1 and P-256 base fields,
the curve constants in that form (b, beta, G), and secp256k1's GLV split
constants (kernel K2, corda_amd/csrc/ecdsa.hip).

Every constant is derived here from the curve parameters (SEC 2 v2, 2.4.1 and
2.4.2) and checked before it is written: the generators against the
Montgomery-2^256 limbs the earlier 8 x 32-bit kernels used, the endomorphism
(lambda^3 == 1 mod n, beta^3 == 1 mod p, [lambda]G == (beta Gx, Gy)), the
lattice basis from extended Euclid on (n, lambda) (a + b lambda == 0 mod n),
and the split bound |k1|, |k2| < 2^129 on random and edge scalars.

    python3 tools/gen_fp29_consts.py           # (re)write the header
    python3 tools/gen_fp29_consts.py --check   # exit 1 if the header is stale
"""
import math
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "corda_amd", "csrc", "fp29_consts.hpp")

P_K1 = 2**256 - 2**32 - 977
N_K1 = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
G_K1 = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
        0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)
P_R1 = 2**256 - 2**224 + 2**192 + 2**96 - 1
N_R1 = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
B_R1 = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
G_R1 = (0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
        0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5)
# secp256k1's endomorphism phi(x, y) = (beta x, y) = [lambda](x, y): a cube root
# of unity in each field (the pairing is checked below)
LAMBDA = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
BETA = 0x7AE96A2B657C07106E64479EAC3434E99CF0497512F58995C1396C28719501EE

# the generators in the Montgomery-2^256 form the earlier 8 x 32-bit kernels stored
OLD_MONT = {
    "K1": ([0x487e2097, 0xd7362e5a, 0x29bc66db, 0x231e2953, 0x33fd129c, 0x979f48c0, 0xe9089f48, 0x9981e643],
           [0xd3dbabe2, 0xb15ea6d2, 0x1f1dc64d, 0x8dfc5d5d, 0xac19c136, 0x70b6b59a, 0xd4a582d6, 0xcf3f851f]),
    "R1": ([0x18a9143c, 0x79e730d4, 0x5fedb601, 0x75ba95fc, 0x77622510, 0x79fb732b, 0xa53755c6, 0x18905f76],
           [0xce95560a, 0xddf25357, 0xba19e45c, 0x8b4ab8e4, 0xdd21f325, 0xd2e88688, 0x25885d85, 0x8571ff18]),
}

R = 2**261
M29 = 2**29 - 1


def limbs29(x, n=9):
    assert 0 <= x < 2**(29 * n)
    return [(x >> (29 * i)) & M29 for i in range(n)]


def words32(x):
    assert 0 <= x < 2**256
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def subkp(p, k):
    """k p (k = 4, 6) as 9 limbs whose limbs 0..7 lie in [2^31 - 4, 2^31 + 2^29): each
    borrows 2^31 (= 4 x 2^29) from the next, so up to three norm subtrahends
    (limbs < 2^29 + 2^15) never take a limb below zero and a norm minuend plus the
    limb stays below 2^32 (fp29.hpp f29_sub2_red / f29_sub3_red)."""
    d = [v for v in limbs29(k * p)]
    for i in range(8):
        d[i] += 2**31
        d[i + 1] -= 4
    assert sum(v << (29 * i) for i, v in enumerate(d)) == k * p
    assert all(2**31 - 4 <= v < 2**31 + 2**29 for v in d[:8]) and 0 <= d[8] < 2**29
    return d


def sub2p(p):
    """2p as 9 limbs whose limbs 0..7 are >= 2^29 - 1 (each borrows 2^29 from the next)."""
    d = [2 * v for v in limbs29(p)]
    for i in range(8):
        d[i] += 2**29
        d[i + 1] -= 1
    assert sum(v << (29 * i) for i, v in enumerate(d)) == 2 * p
    assert all(2**29 - 1 <= v < 2**31 for v in d[:8]) and 0 <= d[8] < 2**29
    return d


def minv29(p):
    return (-pow(p, -1, 2**29)) % 2**29


def ec_add(P, Q, p, a):
    if P is None:
        return Q
    if Q is None:
        return P
    if P[0] == Q[0] and (P[1] + Q[1]) % p == 0:
        return None
    if P == Q:
        lam = (3 * P[0] * P[0] + a) * pow(2 * P[1], -1, p) % p
    else:
        lam = (Q[1] - P[1]) * pow(Q[0] - P[0], -1, p) % p
    x = (lam * lam - P[0] - Q[0]) % p
    return (x, (lam * (P[0] - x) - P[1]) % p)


def ec_mul(k, P, p, a):
    acc = None
    for bit in bin(k)[2:]:
        acc = ec_add(acc, acc, p, a)
        if bit == "1":
            acc = ec_add(acc, P, p, a)
    return acc


def glv_basis(n, lam):
    """Short basis of {(a, b): a + b lam == 0 mod n} by extended Euclid on (n, lam)
    (Gallant-Lambert-Vanstone 2001; Guide to ECC, Alg. 3.74)."""
    s = math.isqrt(n)
    r0, r1, t0, t1 = n, lam, 0, 1
    while r1 >= s:
        q = r0 // r1
        r0, r1, t0, t1 = r1, r0 - q * r1, t1, t0 - q * t1
    q = r0 // r1
    r2, t2 = r0 - q * r1, t0 - q * t1
    a1, b1 = r1, -t1
    a2, b2 = (r0, -t0) if r0 * r0 + t0 * t0 <= r2 * r2 + t2 * t2 else (r2, -t2)
    return a1, b1, a2, b2


A1, B1, A2, B2 = glv_basis(N_K1, LAMBDA)
G1 = (2**384 * B2 + N_K1 // 2) // N_K1     # round(2^384 b2 / n)
G2 = (2**384 * -B1 + N_K1 // 2) // N_K1    # round(2^384 (-b1) / n)


def glv_split(k):
    """ecdsa.hip glv_split, step for step: k == r1 + r2 lambda (mod n)."""
    c1 = (k * G1 + (1 << 383)) >> 384
    c2 = (k * G2 + (1 << 383)) >> 384
    r2 = (c1 * (-B1 % N_K1) + c2 * (-B2 % N_K1)) % N_K1
    r1 = (r2 * (-LAMBDA % N_K1) + k) % N_K1
    return r1, r2


def signed_mag(r, n):
    """split_sign in ecdsa.hip: negative when bit 255 is set."""
    return (n - r, True) if r >> 255 else (r, False)


def check():
    for name, p, (gx, gy) in (("K1", P_K1, G_K1), ("R1", P_R1, G_R1)):
        assert words32(gx * 2**256 % p) == OLD_MONT[name][0], name
        assert words32(gy * 2**256 % p) == OLD_MONT[name][1], name
        assert p % 4 == 3
    assert (G_K1[1]**2 - G_K1[0]**3 - 7) % P_K1 == 0
    assert (G_R1[1]**2 - G_R1[0]**3 + 3 * G_R1[0] - B_R1) % P_R1 == 0
    assert 2**256 - P_K1 == 2**32 + 977                        # f29_red, secp256k1
    assert 2**256 - P_R1 == 2**224 - 2**192 - 2**96 + 1        # f29_red, P-256
    assert minv29(P_R1) == 1 and minv29(P_K1) != 1
    assert pow(LAMBDA, 3, N_K1) == 1 and LAMBDA != 1
    assert pow(BETA, 3, P_K1) == 1 and BETA != 1
    assert ec_mul(LAMBDA, G_K1, P_K1, 0) == (BETA * G_K1[0] % P_K1, G_K1[1])
    for a, b in ((A1, B1), (A2, B2)):
        assert (a + b * LAMBDA) % N_K1 == 0 and a.bit_length() <= 129 and abs(b).bit_length() <= 129
    rng = random.Random(1)
    edge = [0, 1, 2, N_K1 - 1, N_K1 - 2, N_K1 // 2, N_K1 // 2 + 1, LAMBDA, N_K1 - LAMBDA, 2**128, 2**128 - 1,
            2**255, 2**256 % N_K1, A1, A2, N_K1 - A1]
    worst = 0
    for k in edge + [rng.randrange(N_K1) for _ in range(20000)]:
        r1, r2 = glv_split(k)
        assert (r1 + r2 * LAMBDA - k) % N_K1 == 0
        for r in (r1, r2):
            worst = max(worst, signed_mag(r, N_K1)[0].bit_length())
    assert worst <= 129, worst
    return worst


HEADER = """\
// Generated by tools/gen_fp29_consts.py: do not edit (re-run the script).
// Radix-2^29 Montgomery constants (R = 2^261) of the secp256k1 / P-256 base
// fields for fp29.hpp, curve constants in that form (b, beta, G: Montgomery,
// canonical), and the secp256k1 GLV split constants (8 x 32-bit limbs, scalar
// field mod n; *M = Montgomery-2^256 form for mont_mul<K1N>).
#pragma once
#include <stdint.h>

#ifndef CDEV
#define CDEV __device__ __forceinline__
#endif

#define F29_LIMBS(name, a0, a1, a2, a3, a4, a5, a6, a7, a8)                                              \\
  CDEV static constexpr uint32_t name(int i) {                                                           \\
    return i == 0 ? a0 : i == 1 ? a1 : i == 2 ? a2 : i == 3 ? a3 : i == 4 ? a4 : i == 5 ? a5 : i == 6 ? a6 \\
         : i == 7 ? a7 : a8;                                                                             \\
  }
#define W8_LIMBS(name, a0, a1, a2, a3, a4, a5, a6, a7)                                                   \\
  CDEV static constexpr uint32_t name(int i) {                                                           \\
    return i == 0 ? a0 : i == 1 ? a1 : i == 2 ? a2 : i == 3 ? a3 : i == 4 ? a4 : i == 5 ? a5 : i == 6 ? a6 \\
         : a7;                                                                                           \\
  }

namespace cordahip {
"""


def _hex(vals):
    return ", ".join("0x%08xu" % v for v in vals)


def emit_field(name, p, kred, consts, comment):
    out = ["// %s" % comment, "struct %s {" % name]
    out.append("  F29_LIMBS(m, %s)" % _hex(limbs29(p)))
    out.append("  F29_LIMBS(sub2p, %s)" % _hex(sub2p(p)))
    out.append("  F29_LIMBS(sub4p, %s)" % _hex(subkp(p, 4)))
    out.append("  F29_LIMBS(sub6p, %s)" % _hex(subkp(p, 6)))
    out.append("  F29_LIMBS(r2, %s)  // R^2 mod p" % _hex(limbs29(R * R % p)))
    out.append("  F29_LIMBS(one, %s)  // R mod p" % _hex(limbs29(R % p)))
    for tag, v in consts:
        out.append("  F29_LIMBS(%s, %s)" % (tag, _hex(limbs29(v * R % p))))
    out.append("  static constexpr uint32_t kMinv = 0x%08xu;  // -p^-1 mod 2^29" % minv29(p))
    out.append("  static constexpr bool kMinvOne = %s;" % ("true" if minv29(p) == 1 else "false"))
    out.append("  static constexpr int kRed = %d;" % kred)
    out.append("};")
    return "\n".join(out)


def emit_w8(name, v, comment):
    return "struct %s {  // %s\n  W8_LIMBS(limb, %s)\n};" % (name, comment, _hex(words32(v)))


def render():
    parts = [HEADER]
    parts.append(emit_field("K1F", P_K1, 1, [("bm", 7), ("betam", BETA), ("gxm", G_K1[0]), ("gym", G_K1[1])],
                            "secp256k1 base field, p = 2^256 - 2^32 - 977"))
    parts.append(emit_field("R1F", P_R1, 2, [("bm", B_R1), ("betam", 0), ("gxm", G_R1[0]), ("gym", G_R1[1])],
                            "P-256 base field, p = 2^256 - 2^224 + 2^192 + 2^96 - 1"))
    parts.append(emit_w8("K1G1", G1, "round(2^384 b2 / n)"))
    parts.append(emit_w8("K1G2", G2, "round(2^384 (-b1) / n)"))
    parts.append(emit_w8("K1MB1M", (-B1) * 2**256 % N_K1, "-b1, Montgomery form mod n"))
    parts.append(emit_w8("K1MB2M", (-B2) * 2**256 % N_K1, "-b2, Montgomery form mod n"))
    parts.append(emit_w8("K1MLamM", (-LAMBDA) * 2**256 % N_K1, "-lambda, Montgomery form mod n"))
    parts.append("}  // namespace cordahip\n")
    return "\n\n".join(parts)


def main():
    worst = check()
    text = render()
    if "--check" in sys.argv:
        with open(OUT) as f:
            if f.read() != text:
                print("fp29_consts.hpp is stale: re-run tools/gen_fp29_consts.py")
                sys.exit(1)
        print("fp29_consts.hpp up to date (GLV split max magnitude: %d bits)" % worst)
        return
    with open(OUT, "w") as f:
        f.write(text)
    print("wrote %s (GLV split max magnitude: %d bits)" % (OUT, worst))


if __name__ == "__main__":
    main()
