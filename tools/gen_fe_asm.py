#!/usr/bin/env python3
"""Generate corda_amd/csrc/fe25519_asm.hpp: GF(2^255-19) products of TWO,
THREE or FOUR independent operand pairs as one gfx950 inline-asm block each
(fe_mul2, fe_sq2, fe_mul3, fe_mul4, fe_sq4), plus the outer-product blocks
fe_mul3x / fe_mul4x of the formulas' output stage, in the radix-2^25.5
representation of fe25519.hpp.

Why asm: the column accumulation wants the incoming carry as the addend of the
column's first v_mad_u64_u32, so carries cost no instruction. LLVM re-associates
such a chain ((carry + p0) + p1 ... -> (p0 + ... + p9) + carry) and pays one
64-bit add per column (v_lshl_add_u64, a 4-cycle VOP3 on gfx950: 10 per
product, ~8% of a product's issue cycles; tools/microbench/valu_rates.hip). A
carry-chained column is a dependent chain (v_mad_u64_u32 waits ~12 cycles for
its predecessor), so independent products are interleaved instruction by
instruction. Two chains per wave at two waves per SIMD still leave the pair
~25% above its issue cost (profiles/r02_fe_asm_check.jsonl: ~5.2 cycles per
instruction against ~4.1); the group formulas have four independent products
per stage (doubling: X^2, Y^2, Z^2, (X+Y)^2; additions: four, then three or
four), so they use 3- and 4-chain blocks.

The arithmetic is exactly fe25519.hpp's carry-chained fe_mul / fe_sq (same
column terms in the same order, same masks and shifts), so the results are
bit-identical; tools/microbench/fe_asm_check.hip compares them on the GPU.

Run: python3 tools/gen_fe_asm.py  (rewrites the header)
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "corda_amd", "csrc", "fe25519_asm.hpp")
MASK = {0: "0x3ffffff", 1: "0x1ffffff"}  # even limbs 26 bits, odd 25
# The two column accumulators live in fixed VGPR pairs (declared clobbered):
# the limb mask reads the pair's low register, which an operand constraint
# cannot name (FE_ASM_ACC_CLOBBERS in the header); the compiler allocates
# everything else around them.
ACC = ("v[160:161]", "v[162:163]", "v[164:165]", "v[166:167]")
ACC_LO = ("v160", "v162", "v164", "v166")


def bits(k):
    return 25 if k & 1 else 26


def mul_terms(k):
    """(a, b) operand names of column k of f*g, in fe25519.hpp's order."""
    out = []
    for i in range(10):
        j = (k - i + 10) % 10
        wrap = i + j >= 10
        oo = (i & 1) and (j & 1)
        out.append(("f2_%d" % i if oo else "f_%d" % i, "g19_%d" % j if wrap else "g_%d" % j))
    return out


def sq_terms(k):
    out = []
    for i in range(10):
        j = (k - i + 10) % 10
        if j < i:
            continue
        wrap = i + j >= 10
        oo = (i & 1) and (j & 1)
        mult = (2 if i < j else 1) * (2 if oo else 1)
        a = {1: "f_%d", 2: "f2_%d", 4: "f4_%d"}[mult] % i
        out.append((a, "f19_%d" % j if wrap else "f_%d" % j))
    return out


def gen(kind, n):
    """One asm statement for n products; operand names carry a product suffix."""
    terms = [mul_terms(k) if kind == "mul" else sq_terms(k) for k in range(10)]
    need = sorted({x for col in terms for t in col for x in t})
    lines = []
    P = range(n)
    # scaled operands: f2 = 2 f, f4 = 4 f, g19 / f19 = 19 x
    for p in P:
        for nm in need:
            base, idx = nm.split("_")
            src = ("g_%s" % idx) if base == "g19" else ("f_%s" % idx)
            # doublings as adds: v_add_u32 issues at ~2.3 cycles per wave64
            # instruction, v_lshlrev_b32 at ~4.0 (profiles/r02_valu_rates.jsonl)
            if base == "f2":
                lines.append("v_add_u32 %%[%s%d], %%[%s%d], %%[%s%d]" % (nm, p, src, p, src, p))
            elif base == "f4" and ("f2_" + idx) in need:  # sorted: f2_i is already there
                lines.append("v_add_u32 %%[%s%d], %%[f2_%s%d], %%[f2_%s%d]" % (nm, p, idx, p, idx, p))
            elif base == "f4":
                lines.append("v_lshlrev_b32 %%[%s%d], 2, %%[%s%d]" % (nm, p, src, p))
            elif base in ("g19", "f19"):
                lines.append("v_mul_lo_u32 %%[%s%d], %%[%s%d], 19" % (nm, p, src, p))
    for k in range(10):
        col = terms[k]
        for t, (a, b) in enumerate(col):
            for p in P:
                addend = ("0" if k == 0 else "%%[c%d]" % p) if t == 0 else ACC[p]
                lines.append("v_mad_u64_u32 %s, vcc, %%[%s%d], %%[%s%d], %s" % (ACC[p], a, p, b, p, addend))
        for p in P:
            lines.append("v_and_b32 %%[r%d_%d], %s, %s" % (p, k, MASK[k & 1], ACC_LO[p]))
            lines.append("v_lshrrev_b64 %%[c%d], %d, %s" % (p, bits(k), ACC[p]))
    scaled = [nm for nm in need if nm.split("_")[0] in ("f2", "f4", "g19", "f19")]
    return lines, scaled


def asm_block(kind, n):
    lines, scaled = gen(kind, n)
    body = "\n".join('        "%s\\n"' % l for l in lines)
    outs = []
    for p in range(n):
        outs += ['[r%d_%d] "=&v"(o%d.v[%d])' % (p, k, p, k) for k in range(10)]
        outs += ['[c%d] "=&v"(c%d)' % (p, p)]
        outs += ['[%s%d] "=&v"(t%d_%s)' % (nm, p, p, nm) for nm in scaled]
    ins = []
    for p in range(n):
        ins += ['[f_%d%d] "v"(f%d.v[%d])' % (k, p, p, k) for k in range(10)]
        if kind == "mul":
            ins += ['[g_%d%d] "v"(g%d.v[%d])' % (k, p, p, k) for k in range(10)]
    decl = "\n".join("  uint32_t %s;" % ", ".join("t%d_%s" % (p, nm) for nm in scaled) for p in range(n))
    return body, ",\n        ".join(outs), ",\n        ".join(ins), decl


# Outer-product blocks: the formulas' output stage X = F E, Y = H G, Z = F G,
# T = H E is {F, H} x {E, G}, so each operand's scaled copies (2x odd limbs of
# an f-operand, 19x of a g-operand) are made once and shared by the two products
# that read it: 18 v_mul_lo_u32 + 10 v_add_u32 per block instead of 36 + 20 (4
# products) or 27 + 15 (3). Product p is F[fi] * G[gi] over column terms
# mul_terms(k), the same multiset of integer terms as the f/g-swapped product,
# so every column value and hence the carry-chained result is bit-identical.
OUTER = ((0, 0), (1, 1), (0, 1), (1, 0))  # (fi, gi): F0 G0, F1 G1, F0 G1, F1 G0
FSET, GSET = "ab", "cd"


def gen_outer(n):
    terms = [mul_terms(k) for k in range(10)]
    need = sorted({x for col in terms for t in col for x in t})
    lines = []
    scaled = []
    for nm in need:
        base, idx = nm.split("_")
        if base == "f2":
            for fs in FSET:
                lines.append("v_add_u32 %%[f2_%s%s], %%[f_%s%s], %%[f_%s%s]" % (idx, fs, idx, fs, idx, fs))
                scaled.append("f2_%s%s" % (idx, fs))
        elif base == "g19":
            for gs in GSET:
                lines.append("v_mul_lo_u32 %%[g19_%s%s], %%[g_%s%s], 19" % (idx, gs, idx, gs))
                scaled.append("g19_%s%s" % (idx, gs))
    P = range(n)
    for k in range(10):
        for t, (a, b) in enumerate(terms[k]):
            for p in P:
                fi, gi = OUTER[p]
                addend = ("0" if k == 0 else "%%[c%d]" % p) if t == 0 else ACC[p]
                lines.append("v_mad_u64_u32 %s, vcc, %%[%s%s], %%[%s%s], %s" % (ACC[p], a, FSET[fi], b, GSET[gi], addend))
        for p in P:
            lines.append("v_and_b32 %%[r%d_%d], %s, %s" % (p, k, MASK[k & 1], ACC_LO[p]))
            lines.append("v_lshrrev_b64 %%[c%d], %d, %s" % (p, bits(k), ACC[p]))
    return lines, scaled


def outer_block(n):
    lines, scaled = gen_outer(n)
    body = "\n".join('        "%s\\n"' % l for l in lines)
    outs = []
    for p in range(n):
        outs += ['[r%d_%d] "=&v"(o%d.v[%d])' % (p, k, p, k) for k in range(10)]
        outs += ['[c%d] "=&v"(c%d)' % (p, p)]
    outs += ['[%s] "=&v"(t_%s)' % (nm, nm) for nm in scaled]
    ins = []
    for j, fs in enumerate(FSET):
        ins += ['[f_%d%s] "v"(f%d.v[%d])' % (k, fs, j, k) for k in range(10)]
    for j, gs in enumerate(GSET):
        ins += ['[g_%d%s] "v"(g%d.v[%d])' % (k, gs, j, k) for k in range(10)]
    decl = "  uint32_t %s;" % ", ".join("t_%s" % nm for nm in scaled)
    sig = "CDEV void fe_mul%dx(%s, const fe& f0, const fe& f1, const fe& g0, const fe& g1)" % (
        n, ", ".join("fe& r%d" % p for p in range(n)))
    return '''// r0 = f0 g0, r1 = f1 g1, r2 = f0 g1%s (shared scaled operands)
%s {
  fe %s;
  uint64_t %s;
%s
  asm(
%s
      : %s
      : %s
      : "vcc", %s);
%s
%s
}
''' % (", r3 = f1 g0" if n == 4 else "", sig, ", ".join("o%d" % p for p in range(n)),
       ", ".join("c%d" % p for p in range(n)), decl, body, ",\n        ".join(outs), ",\n        ".join(ins),
       CLOBBERS[n], "\n".join("  fe_fold_top(o%d, c%d);" % (p, p) for p in range(n)),
       "\n".join("  r%d = o%d;" % (p, p) for p in range(n)))


HEADER = '''// GENERATED by tools/gen_fe_asm.py -- do not edit; re-run the script.
//
// GF(2^255-19) products of two, three or four independent operand pairs, each
// as ONE gfx950 inline-asm block: carry-chained columns (the incoming carry is
// the addend of the column's first v_mad_u64_u32, so carries cost no add), the
// products' chains interleaved instruction by instruction (a dependent
// v_mad_u64_u32 waits for its predecessor; more chains per wave hide more of
// that latency). Bit-identical to fe25519.hpp's carry-chained fe_mul / fe_sq
// (checked by tools/microbench/fe_asm_check.hip); same operand bounds.
#pragma once
#include "fe25519.hpp"

// the accumulators' fixed VGPRs (v160..v167): see tools/gen_fe_asm.py
#define FE_ASM_ACC_CLOBBERS "v160", "v161", "v162", "v163"
#define FE_ASM_ACC_CLOBBERS3 FE_ASM_ACC_CLOBBERS, "v164", "v165"
#define FE_ASM_ACC_CLOBBERS4 FE_ASM_ACC_CLOBBERS3, "v166", "v167"

namespace cordahip {
'''

CLOBBERS = {2: "FE_ASM_ACC_CLOBBERS", 3: "FE_ASM_ACC_CLOBBERS3", 4: "FE_ASM_ACC_CLOBBERS4"}


def signature(kind, n):
    if kind == "mul":
        args = ", ".join("fe& r%d, const fe& f%d, const fe& g%d" % (p, p, p) for p in range(n))
    else:
        args = ", ".join("fe& r%d, const fe& f%d" % (p, p) for p in range(n))
    return "CDEV void fe_%s%d(%s)" % (kind, n, args)


def render():
    parts = [HEADER]
    for kind, n in (("mul", 2), ("sq", 2), ("mul", 3), ("mul", 4), ("sq", 4)):
        body, outs, ins, decl = asm_block(kind, n)
        parts.append('''%s {
  fe %s;
  uint64_t %s;
%s
  asm(
%s
      : %s
      : %s
      : "vcc", %s);
%s
%s
}
''' % (signature(kind, n), ", ".join("o%d" % p for p in range(n)), ", ".join("c%d" % p for p in range(n)),
       decl, body, outs, ins, CLOBBERS[n],
       "\n".join("  fe_fold_top(o%d, c%d);" % (p, p) for p in range(n)),
       "\n".join("  r%d = o%d;" % (p, p) for p in range(n))))
    for n in (3, 4):
        parts.append(outer_block(n))
    parts.append("}  // namespace cordahip\n")
    return "\n".join(parts)


def main():
    with open(OUT, "w") as f:
        f.write(render())
    print("wrote", OUT)


if __name__ == "__main__":
    main()
