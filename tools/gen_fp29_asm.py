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
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "corda_amd", "csrc", "fp29_asm.hpp")
M29 = "0x1fffffff"
ACC = ("v[160:161]", "v[162:163]")
ACC_LO = ("v160", "v162")

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_fp29_consts as fc  # noqa: E402

CURVES = {
    # p limbs (radix 2^29), -p^-1 mod 2^29 (None: 1)
    "k1": ([0x1ffffc2f, 0x1ffffff7, 0x1fffffff, 0x1fffffff, 0x1fffffff, 0x1fffffff, 0x1fffffff, 0x1fffffff,
            0x00ffffff], 0x12253531),
    "r1": ([0x1fffffff, 0x1fffffff, 0x1fffffff, 0x000001ff, 0x00000000, 0x00000000, 0x00040000, 0x1fe00000,
            0x00ffffff], None),
}


SUBKP = {c: {k: fc.subkp(pv, k) for k in (4, 6)} for c, pv in (("k1", fc.P_K1), ("r1", fc.P_R1))}


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


def product_terms(kind, curve, nsub=0):
    """fp29.hpp's f29_mul / f29_sqr schedule for one product: a list of steps per
    column. Steps: ('mad', a, b) | ('madq', j, const) (q_j * const) | ('madqn', j)
    (+ qn_j) | ('addM',) | ('minus1',) | ('q', k) | ('sub', i) | ('out', k) |
    ('shift',) | ('top',). With nsub subtrahends, ('sub', i) adds kp_i - sum s_i
    (limb i of kp - s0 - s1 ..., every limb >= 0) into output column 9 + i and
    the top: the REDC then returns red(ab) + kp - sum s unnormalised at the top,
    for f29_fold (fp29.hpp f29_mul_sub)."""
    cols = []
    for k in range(17):
        st = []
        lo, hi = max(0, k - 8), min(k, 8)
        if kind in ("mul", "mul2"):
            for j in range(lo, hi + 1):
                st.append(("mad", "a%d" % j, "b%d" % (k - j)))
            if kind == "mul2":  # + c d in the same columns: one REDC for the sum
                for j in range(lo, hi + 1):
                    st.append(("mad", "c%d" % j, "d%d" % (k - j)))
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
            if nsub:
                st.append(("sub", k - 9))
            st.append(("out", k - 9))
        st.append(("shift",))
        cols.append(st)
    cols.append(([("sub", 8)] if nsub else []) + [("top",)])
    return cols


def sub_k(nsub):
    """The multiple of p added with nsub norm subtrahends: 4p for one or two
    (sub4p's limbs 0..7 exceed two norm limbs), 6p for three."""
    return 4 if nsub <= 2 else 6


def expand(kind, p, curve, subs=()):
    """Asm lines of one product p (0/1) as a list of per-column instruction lists.
    subs: the subtrahends' operand names as format strings of the limb index
    ("s0_0_{}": an input f29; "t{}_0": product 0's own output limbs)."""
    cols = []
    skp = SUBKP[curve][sub_k(len(subs))] if subs else None
    for st in product_terms(kind, curve, len(subs)):
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
            elif s[0] == "sub":
                i = s[1]
                lines.append("v_sub_u32 %%[x_%d], 0x%08x, %%[%s]" % (p, skp[i], subs[0].format(i)))
                for sb in subs[1:]:
                    lines.append("v_sub_u32 %%[x_%d], %%[x_%d], %%[%s]" % (p, p, sb.format(i)))
                if i < 8:
                    lines.append("v_mad_u64_u32 %s, vcc, %%[x_%d], 1, %s" % (ACC[p], p, ACC[p]))
            elif s[0] == "shift":
                lines.append("v_lshrrev_b64 %s, 29, %s" % (ACC[p], ACC[p]))
            elif s[0] == "out":
                lines.append("v_and_b32 %%[t%d_%d], %s, %s" % (s[1], p, M29, ACC_LO[p]))
            elif s[0] == "top":
                if subs:  # the top limb wraps mod 2^32 like the C version's
                    lines.append("v_add_u32 %%[t8_%d], %%[x_%d], %s" % (p, p, ACC_LO[p]))
                else:
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


def sub_names(subs, p):
    """Operand-name formats of product p's subtrahends: 'e' = an input f29
    (s<p><j>), 'o' = product 0's output (the pair's partner, computed column by
    column ahead of it)."""
    out = []
    for j, kind in enumerate(subs):
        out.append("s%d%d_{}" % (p, j) if kind == "e" else "t{}_0")
    return out


def check_order(lines):
    """Every operand read by a v_sub_u32 of a subtrahend that is product 0's
    output is written earlier in the block."""
    written = set()
    for l in lines:
        op, rest = l.split(" ", 1)
        args = [x.strip() for x in rest.split(",")]
        if op == "v_sub_u32":
            for x in args[1:]:
                if x.startswith("%[t") and x.endswith("_0]"):
                    assert x in written, "subtrahend %s read before it is written" % x
        if args[0].startswith("%["):
            written.add(args[0])


def gen(curve, kinds, subs=((), ())):
    m, minv = CURVES[curve]
    lines = []
    # the first column of each product starts from 0: rewrite its first mad's addend
    per = []
    for p, kind in enumerate(kinds):
        cols = expand(kind, p, curve, sub_names(subs[p], p))
        first = cols[0][0]
        cols[0][0] = first[: first.rfind(",")] + ", 0"
        if kind == "sqr":
            # 2a as an add: v_add_u32 issues at ~2.3 cycles, v_lshlrev_b32 at ~4.0
            cols[0] = ["v_add_u32 %%[a2_%d_%d], %%[a%d_%d], %%[a%d_%d]" % (j, p, j, p, j, p) for j in range(8)] + cols[0]
        per.append(cols)
    lines = interleave(per[0], per[1]) if len(per) == 2 else [l for col in per[0] for l in col]
    check_order(lines)
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
        if subs[p]:
            outs.append('[x_%d] "=&v"(x%d)' % (p, p))
            decl.append("uint32_t x%d;" % p)
        ins += ['[a%d_%d] "v"(a%d.v[%d])' % (k, p, p, k) for k in range(9)]
        if kind in ("mul", "mul2"):
            ins += ['[b%d_%d] "v"(b%d.v[%d])' % (k, p, p, k) for k in range(9)]
        if kind == "mul2":
            ins += ['[c%d_%d] "v"(c%d.v[%d])' % (k, p, p, k) for k in range(9)]
            ins += ['[d%d_%d] "v"(d%d.v[%d])' % (k, p, p, k) for k in range(9)]
        for j, sk in enumerate(subs[p]):
            if sk == "e":
                ins += ['[s%d%d_%d] "v"(s%d%d.v[%d])' % (p, j, k, p, j, k) for k in range(9)]
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
//
// The *_sub variants fold the formulas' "product minus norm subtrahends" steps
// into the REDC (fp29.hpp f29_sub*_red after a product): output column 9 + i
// also accumulates limb i of kp - s0 - s1 ... (k = 4, or 6 for three
// subtrahends; every such limb >= 0), so the carry pass the REDC already makes
// is the subtraction's too, and f29_fold brings the top below 2p: the same
// value as the product followed by f29_sub*_red.
#pragma once
#include "fp29.hpp"
#include "fp29_consts.hpp"

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
# products with folded subtrahends (name, kinds, subtrahends per product, signature):
#   mul_mul_s1s1: r0 = a0 b0 - s00, r1 = a1 b1 - s10      (jmadd: H, R)
#   sqr_mul_s2:   r0 = a0^2 - s00 - s01, r1 = a1 b1      (jdbl: X3 and Z3)
#   sqr_mul_s3:   r0 = a0^2 - s00 - s01 - s02, r1 = a1 b1 (jmadd: X3 and Y1 J)
#   sqr_mul_o2:   r0 = a0^2, r1 = a1 b1 - 2 r0           (P-256 jdbl: 4 gamma^2, Y3)
#   mul_s2:       r0 = a0 b0 - s00 - s01                  (Y3 of jmadd, secp256k1 jdbl)
SUB_FUNCS = (
    (("mul", "mul"), "mul_mul_s1s1", (("e",), ("e",)),
     "f29& r0, const f29& a0, const f29& b0, const f29& s00, f29& r1, const f29& a1, const f29& b1, const f29& s10"),
    (("sqr", "mul"), "sqr_mul_s2", (("e", "e"), ()),
     "f29& r0, const f29& a0, const f29& s00, const f29& s01, f29& r1, const f29& a1, const f29& b1"),
    (("sqr", "mul"), "sqr_mul_s3", (("e", "e", "e"), ()),
     "f29& r0, const f29& a0, const f29& s00, const f29& s01, const f29& s02, f29& r1, const f29& a1, const f29& b1"),
    (("sqr", "mul"), "sqr_mul_o2", ((), ("o", "o")), "f29& r0, const f29& a0, f29& r1, const f29& a1, const f29& b1"),
    (("mul",), "mul_s2", (("e", "e"),), "f29& r0, const f29& a0, const f29& b0, const f29& s00, const f29& s01"),
    #   mul2:         r0 = a0 b0 + c0 d0, ONE REDC             (jmadd: Y3 = r (V - X3) + Y1 (4p - 2J))
    #   sqr_s3:       r0 = a0^2 - s00 - s01 - s02              (jmadd: X3, now unpaired)
    (("mul2",), "mul2", ((),), "f29& r0, const f29& a0, const f29& b0, const f29& c0, const f29& d0"),
    (("sqr",), "sqr_s3", (("e", "e", "e"),), "f29& r0, const f29& a0, const f29& s00, const f29& s01, const f29& s02"),
    #   sqr_sqr_s2s2: r0 = a0^2 - s00 - s01, r1 = a1^2 - s10 - s11  (P-256 jdbl: X3, Z3)
    #   sqr_mul_s2s2: r0 = a0^2 - s00 - s01, r1 = a1 b1 - s10 - s11 (jmadd: Z3, Y3)
    (("sqr", "sqr"), "sqr_sqr_s2s2", (("e", "e"), ("e", "e")),
     "f29& r0, const f29& a0, const f29& s00, const f29& s01, f29& r1, const f29& a1, const f29& s10, const f29& s11"),
    (("sqr", "mul"), "sqr_mul_s2s2", (("e", "e"), ("e", "e")),
     "f29& r0, const f29& a0, const f29& s00, const f29& s01, f29& r1, const f29& a1, const f29& b1, const f29& s10, "
     "const f29& s11"),
)


def render():
    """The header's full text."""
    parts = [HEADER]
    for curve in ("k1", "r1"):
        fty = "K1F" if curve == "k1" else "R1F"
        funcs = [(k, n, ((),) * len(k), sg) for k, n, sg in FUNCS] + [(k, n, sb, sg) for k, n, sb, sg in SUB_FUNCS]
        for kinds, name, subs, sig in funcs:
            body, outs, ins, decl = gen(curve, kinds, subs)
            n = len(kinds)
            fin = []
            for p in range(n):
                if subs[p]:  # limbs 0..7 normalised by the REDC, the top still to fold
                    fin.append("  f29_fold<%s>(o%d, o%d.v[8]);" % (fty, p, p))
                fin.append("  r%d = o%d;" % (p, p))
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
''' % (name, curve, sig, ", ".join("o%d" % p for p in range(n)), decl, body, outs, ins, "\n".join(fin)))
    parts.append("}  // namespace cordahip\n")
    return "\n".join(parts)


def main():
    with open(OUT, "w") as f:
        f.write(render())
    print("wrote", OUT)


if __name__ == "__main__":
    main()
