#!/usr/bin/env python3
"""Generate corda_amd/csrc/fp29_asm.hpp: radix-2^29 Montgomery products
(fp29.hpp f29_mul / f29_sqr, R = 2^261) of TWO independent operand pairs as one
gfx950 inline-asm block, per curve (secp256k1 "k1", P-256 "r1") and per pair
shape (mul+mul, sqr+sqr, sqr+mul), plus single mul / sqr blocks.

Same reason as tools/gen_fe_asm.py: product scanning keeps ONE running 64-bit
accumulator per product (column k's sum continues from column k-1's, shifted
right by 29), which LLVM re-associates at a cost of one 64-bit add per column
(17 per product); here the accumulator is the v_mad_u64_u32 addend throughout
and the two products' chains are interleaved instruction by instruction.

The terms, their order and every mask, shift and q computation are exactly
fp29.hpp's (its special-form REDC: P-256 4 q terms per column digit and no m0
term, secp256k1 4 q terms plus the (2^29 - 1 - q) bias terms), so the results
are bit-identical to fp29.hpp and to a generic REDC
(tests/test_fp29_asm.py emulates the header on the CPU,
tools/microbench/fp29_asm_check.hip compares it on the GPU). Constants are
SGPR operands.

Run: python3 tools/gen_fp29_asm.py  (rewrites the header)
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "corda_amd", "csrc", "fp29_asm.hpp")
M29 = "0x1fffffff"
ACC = ("v[160:161]", "v[162:163]")
ACC_LO = ("v160", "v162")

CURVES = {
    # p limbs (radix 2^29), -p^-1 mod 2^29 (None: 1)
    "k1": ([0x1ffffc2f, 0x1ffffff7, 0x1fffffff, 0x1fffffff, 0x1fffffff, 0x1fffffff, 0x1fffffff, 0x1fffffff,
            0x00ffffff], 0x12253531),
    "r1": ([0x1fffffff, 0x1fffffff, 0x1fffffff, 0x000001ff, 0x00000000, 0x00000000, 0x00040000, 0x1fe00000,
            0x00ffffff], None),
}


def redc_terms(curve, k):
    """fp29.hpp f29_redc_terms: the q terms (and bias constants) of column k."""
    st = []
    if curve == "k1":
        if 1 <= k <= 9:
            st.append(("madq", k - 1, "m1"))
        if 2 <= k <= 10:
            st.append(("madqn", k - 2))
        if 11 <= k <= 15:
            st.append(("addM",))
        if k == 16:
            st.append(("minus1",))
        if k >= 8:
            st.append(("madq", k - 8, "c24"))
    else:
        if 3 <= k <= 11:
            st.append(("madq", k - 3, "c9"))
        if 6 <= k <= 14:
            st.append(("madq", k - 6, "c18"))
        if 7 <= k <= 15:
            st.append(("madq", k - 7, "m7"))
        if k >= 8:
            st.append(("madq", k - 8, "m8"))
    return st


def product_terms(kind, curve):
    """fp29.hpp's f29_mul / f29_sqr schedule for one product: a list of steps per
    column. Steps: ('mad', a, b) | ('madq', j, const) (q_j * const) | ('madqn', j)
    (+ qn_j) | ('addM',) | ('minus1',) | ('q', k) | ('out', k) | ('shift',) | ('top',)."""
    cols = []
    for k in range(17):
        st = []
        lo, hi = max(0, k - 8), min(k, 8)
        if kind == "mul":
            for j in range(lo, hi + 1):
                st.append(("mad", "a%d" % j, "b%d" % (k - j)))
        else:
            for j in range(lo, hi + 1):
                if 2 * j < k:
                    st.append(("mad", "a2_%d" % j, "a%d" % (k - j)))
            if k % 2 == 0:
                st.append(("mad", "a%d" % (k // 2), "a%d" % (k // 2)))
        st += redc_terms(curve, k)
        if k < 9:
            st.append(("q", k))
        else:
            st.append(("out", k - 9))
        st.append(("shift",))
        cols.append(st)
    cols.append([("top",)])
    return cols


def expand(kind, p, curve):
    """Asm lines of one product p (0/1) as a list of per-column instruction lists."""
    cols = []
    for st in product_terms(kind, curve):
        lines = []
        for s in st:
            if s[0] == "mad":
                lines.append("v_mad_u64_u32 %s, vcc, %%[%s_%d], %%[%s_%d], %s" % (ACC[p], s[1], p, s[2], p, ACC[p]))
            elif s[0] == "madq":
                lines.append("v_mad_u64_u32 %s, vcc, %%[q%d_%d], %%[%s], %s" % (ACC[p], s[1], p, s[2], ACC[p]))
            elif s[0] == "madqn":
                lines.append("v_mad_u64_u32 %s, vcc, %%[qn%d_%d], 1, %s" % (ACC[p], s[1], p, ACC[p]))
            elif s[0] == "addM":
                lines.append("v_mad_u64_u32 %s, vcc, %%[mask], 1, %s" % (ACC[p], ACC[p]))
            elif s[0] == "minus1":
                lines.append("v_lshl_add_u64 %s, -1, 0, %s" % (ACC[p], ACC[p]))
            elif s[0] == "q":
                k = s[1]
                if curve == "k1":
                    lines.append("v_mul_lo_u32 %%[q%d_%d], %s, %%[minv]" % (k, p, ACC_LO[p]))
                    lines.append("v_and_b32 %%[q%d_%d], %s, %%[q%d_%d]" % (k, p, M29, k, p))
                    lines.append("v_sub_u32 %%[qn%d_%d], %s, %%[q%d_%d]" % (k, p, "0x20000000" if k == 0 else M29, k, p))
                    lines.append("v_mad_u64_u32 %s, vcc, %%[q%d_%d], %%[m0], %s" % (ACC[p], k, p, ACC[p]))
                else:
                    lines.append("v_and_b32 %%[q%d_%d], %s, %s" % (k, p, M29, ACC_LO[p]))
            elif s[0] == "shift":
                lines.append("v_lshrrev_b64 %s, 29, %s" % (ACC[p], ACC[p]))
            elif s[0] == "out":
                lines.append("v_and_b32 %%[t%d_%d], %s, %s" % (s[1], p, M29, ACC_LO[p]))
            elif s[0] == "top":
                lines.append("v_mov_b32 %%[t8_%d], %s" % (p, ACC_LO[p]))
        cols.append(lines)
    return cols


def interleave(c0, c1):
    """Alternate the two products' instruction streams, column by column."""
    out = []
    for a, b in zip(c0, c1):
        n = max(len(a), len(b))
        for i in range(n):
            if i < len(a):
                out.append(a[i])
            if i < len(b):
                out.append(b[i])
    return out


def gen(curve, kinds):
    m, minv = CURVES[curve]
    lines = []
    # the first column of each product starts from 0: rewrite its first mad's addend
    per = []
    for p, kind in enumerate(kinds):
        cols = expand(kind, p, curve)
        first = cols[0][0]
        cols[0][0] = first[: first.rfind(",")] + ", 0"
        if kind == "sqr":
            # 2a as an add: v_add_u32 issues at ~2.3 cycles, v_lshlrev_b32 at ~4.0
            cols[0] = ["v_add_u32 %%[a2_%d_%d], %%[a%d_%d], %%[a%d_%d]" % (j, p, j, p, j, p) for j in range(8)] + cols[0]
        per.append(cols)
    lines = interleave(per[0], per[1]) if len(per) == 2 else [l for col in per[0] for l in col]
    body = "\n".join('        "%s\\n"' % l for l in lines)
    outs, ins = [], []
    decl = []
    for p, kind in enumerate(kinds):
        outs += ['[t%d_%d] "=&v"(o%d.v[%d])' % (k, p, p, k) for k in range(9)]
        outs += ['[q%d_%d] "=&v"(q%d[%d])' % (k, p, p, k) for k in range(9)]
        decl.append("uint32_t q%d[9];" % p)
        if curve == "k1":
            outs += ['[qn%d_%d] "=&v"(qn%d[%d])' % (k, p, p, k) for k in range(9)]
            decl.append("uint32_t qn%d[9];" % p)
        if kind == "sqr":
            outs += ['[a2_%d_%d] "=&v"(a2_%d[%d])' % (j, p, p, j) for j in range(8)]
            decl.append("uint32_t a2_%d[8];" % p)
        ins += ['[a%d_%d] "v"(a%d.v[%d])' % (k, p, p, k) for k in range(9)]
        if kind == "mul":
            ins += ['[b%d_%d] "v"(b%d.v[%d])' % (k, p, p, k) for k in range(9)]
    if curve == "k1":
        consts = [("m0", m[0]), ("m1", m[1]), ("c24", 1 << 24), ("mask", (1 << 29) - 1), ("minv", minv)]
    else:
        consts = [("c9", 1 << 9), ("c18", 1 << 18), ("m7", m[7]), ("m8", m[8])]
    ins += ['[%s] "s"(%du)' % c for c in consts]
    return body, ",\n        ".join(outs), ",\n        ".join(ins), "\n  ".join(decl)


HEADER = '''// GENERATED by tools/gen_fp29_asm.py -- do not edit; re-run the script.
//
// Radix-2^29 Montgomery products (fp29.hpp f29_mul / f29_sqr, special-form
// REDC) of two independent operand pairs, each as ONE gfx950 inline-asm block: the running
// column accumulator is the v_mad_u64_u32 addend throughout (no re-associated
// 64-bit adds), the two products' chains interleaved instruction by
// instruction. Bit-identical to fp29.hpp (tools/microbench/fp29_asm_check.hip).
#pragma once
#include "fp29.hpp"

#ifndef FE_ASM_ACC_CLOBBERS
#define FE_ASM_ACC_CLOBBERS "v160", "v161", "v162", "v163"  // accumulators (tools/gen_fe_asm.py)
#endif

namespace cordahip {
'''


FUNCS = (
    (("mul", "mul"), "mul_mul", "f29& r0, const f29& a0, const f29& b0, f29& r1, const f29& a1, const f29& b1"),
    (("sqr", "sqr"), "sqr_sqr", "f29& r0, const f29& a0, f29& r1, const f29& a1"),
    (("sqr", "mul"), "sqr_mul", "f29& r0, const f29& a0, f29& r1, const f29& a1, const f29& b1"),
    # single products (no partner in the formula): still one asm chain, so the
    # accumulator stays the mad addend (LLVM's version re-associates: +17 adds)
    (("mul",), "mul", "f29& r0, const f29& a0, const f29& b0"),
    (("sqr",), "sqr", "f29& r0, const f29& a0"),
)


def render():
    """The header's full text."""
    parts = [HEADER]
    for curve in ("k1", "r1"):
        for kinds, name, sig in FUNCS:
            body, outs, ins, decl = gen(curve, kinds)
            n = len(kinds)
            parts.append('''CDEV void f29a_%s_%s(%s) {
  f29 %s;
  %s
  asm(
%s
      : %s
      : %s
      : "vcc", FE_ASM_ACC_CLOBBERS);
%s
}
''' % (name, curve, sig, ", ".join("o%d" % p for p in range(n)), decl, body, outs, ins,
       "\n".join("  r%d = o%d;" % (p, p) for p in range(n))))
    parts.append("}  // namespace cordahip\n")
    return "\n".join(parts)


def main():
    with open(OUT, "w") as f:
        f.write(render())
    print("wrote", OUT)


if __name__ == "__main__":
    main()
