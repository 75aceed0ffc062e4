"""CPU check of the generated paired Montgomery products (corda_amd/csrc/fp29_asm.hpp).

The header is emulated instruction by instruction (v_mad_u64_u32, v_mul_lo_u32,
v_and_b32, v_lshrrev_b64, v_lshlrev_b32, v_mov_b32 on 32/64-bit registers) for
random operands within f29_mul's bounds and compared with a restatement of
a generic product-scanning REDC over p's nine limbs (and with a b R^-1 mod p);
every column value is checked to stay in [0, 2^64) at each use. The
GPU-side bit-identity check is tools/microbench/fp29_asm_check.hip.
"""
import os
import random
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "corda_amd", "csrc", "fp29_asm.hpp")
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_fp29_asm  # noqa: E402

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1
M29 = (1 << 29) - 1


def parse_header(text):
    """{function name: (asm lines, {operand name: C expression or int})}"""
    funcs = {}
    for m in re.finditer(r"CDEV void (f29a_\w+)\(.*?\n  asm\(\n(.*?)\n      : (.*?)\n      : (.*?)\n      : ", text, re.S):
        name, body, outs, ins = m.groups()
        lines = [l.strip()[1:-3] for l in body.split("\n")]
        ops = {}
        for o in re.finditer(r'\[(\w+)\] "=?&?([vs])"\(([^)]*)\)', outs + "," + ins):
            expr = o.group(3)
            ops[o.group(1)] = int(expr.rstrip("u")) if expr[0].isdigit() else expr
        funcs[name] = (lines, ops)
    return funcs


def emulate(lines, ops, a, b, subs=None):
    """Run one asm body; a/b: {0: limbs, 1: limbs}; subs: {"s00": limbs, ...};
    returns (r0 limbs, r1 limbs) as the asm leaves them (before any fold)."""
    vals = {}
    for n, e in ops.items():
        if isinstance(e, int):
            vals[n] = e
            continue
        mm = re.fullmatch(r"([ab])([01])\.v\[(\d)\]", e)
        if mm and int(mm.group(2)) in (a if mm.group(1) == "a" else b):
            vals[n] = (a if mm.group(1) == "a" else b)[int(mm.group(2))][int(mm.group(3))]
        ms = re.fullmatch(r"(s\d\d|[cd]0)\.v\[(\d)\]", e)
        if ms:
            vals[n] = subs[ms.group(1)][int(ms.group(2))]
    acc = {"v[160:161]": 0, "v[162:163]": 0}  # exact integers: a wrap is an error

    def val(x):
        x = x.strip()
        if x.startswith("%["):
            return vals[x[2:-1]]
        if x in acc:
            assert 0 <= acc[x] < 1 << 64, "column value out of range"
            return acc[x]
        if x in ("v160", "v162"):
            v = acc["v[%s:%d]" % (x[1:], int(x[1:]) + 1)]
            assert 0 <= v < 1 << 64, "column value out of range"
            return v & M32
        return int(x, 0)

    def dst(x):
        assert x.startswith("%["), x
        return x[2:-1]

    for line in lines:
        op, rest = line.split(" ", 1)
        x = [t.strip() for t in rest.split(",")]
        if op == "v_mad_u64_u32":
            assert x[1] == "vcc"
            acc[x[0]] = val(x[2]) * val(x[3]) + (acc[x[4]] if x[4] in acc else val(x[4]))
        elif op == "v_lshl_add_u64":  # only the bias -1: (-1 << 0) + acc
            assert x[1:3] == ["-1", "0"] and x[3] == x[0]
            acc[x[0]] -= 1
        elif op == "v_mul_lo_u32":
            vals[dst(x[0])] = (val(x[1]) * val(x[2])) & M32
        elif op == "v_and_b32":
            vals[dst(x[0])] = val(x[1]) & val(x[2])
        elif op == "v_sub_u32":  # wraps mod 2^32 (the folded top limb may)
            vals[dst(x[0])] = (val(x[1]) - val(x[2])) & M32
        elif op == "v_lshrrev_b64":
            acc[x[0]] = val(x[2]) >> int(x[1])
        elif op == "v_add_u32":
            vals[dst(x[0])] = (val(x[1]) + val(x[2])) & M32
        elif op == "v_lshlrev_b32":
            vals[dst(x[0])] = (val(x[2]) << int(x[1])) & M32
        elif op == "v_mov_b32":
            vals[dst(x[0])] = val(x[1])
        else:
            raise AssertionError("unexpected instruction " + op)
    out = []
    for p in range(2):
        if "t0_%d" % p in vals:
            out.append([vals["t%d_%d" % (k, p)] for k in range(9)])
    return out


def f29_mul_model(curve, a, b):
    """Generic product-scanning REDC over p's nine limbs (fp29.hpp before the
    special-form reduction; the special form must give the same limbs)."""
    m, minv = gen_fp29_asm.CURVES[curve]
    acc, q, t = 0, [0] * 9, [0] * 9
    for k in range(9):
        for j in range(k):
            acc += a[j] * b[k - j] + q[j] * m[k - j]
        acc += a[k] * b[0]
        q[k] = (((acc & M32) * (minv or 1)) & M32) & M29
        acc += q[k] * m[0]
        assert acc < 1 << 64
        acc >>= 29
    for k in range(9, 17):
        for j in range(k - 8, 9):
            acc += a[j] * b[k - j] + q[j] * m[k - j]
        assert acc < 1 << 64
        t[k - 9] = acc & M29
        acc >>= 29
    t[8] = acc & M32
    return t


def value(limbs):
    return sum(x << (29 * i) for i, x in enumerate(limbs))


def test_header_is_generated():
    with open(HDR) as f:
        assert f.read() == gen_fp29_asm.render(), "re-run tools/gen_fp29_asm.py"


@pytest.mark.parametrize("curve", ["k1", "r1"])
@pytest.mark.parametrize("shape", ["mul_mul", "sqr_sqr", "sqr_mul", "mul", "sqr"])
def test_pairs_match_f29_mul(curve, shape):
    with open(HDR) as f:
        funcs = parse_header(f.read())
    lines, ops = funcs["f29a_%s_%s" % (shape, curve)]
    kinds = shape.split("_")
    m, _ = gen_fp29_asm.CURVES[curve]
    p = value(m)
    rinv = pow(2, -261, p)
    rng = random.Random(hash((curve, shape)) & 0xffff)

    def rnd():  # < 2^257 (< 4p): within f29_mul's operand bounds
        return [rng.getrandbits(29) for _ in range(8)] + [rng.getrandbits(25)]

    loose = 0x4C1BF828  # 2^30.25: f29_mul's loose limb bound (both operands)
    edge = [[M29] * 8 + [(1 << 25) - 1], [0] * 9, [1] + [0] * 8, [loose] * 8 + [1 << 24]]
    for it in range(60):
        a = {0: edge[it] if it < len(edge) else rnd(), 1: rnd()}
        b = {0: rnd(), 1: edge[it] if it < len(edge) else rnd()}
        if it == len(edge) - 1:
            a[1] = b[0] = edge[it]
        for q in range(len(kinds)):
            if kinds[q] == "sqr":
                b[q] = a[q]
        got = emulate(lines, ops, a, b)
        assert len(got) == len(kinds)
        for q in range(len(kinds)):
            want = f29_mul_model(curve, a[q], b[q])
            assert got[q] == want
            assert value(want) % p == value(a[q]) * value(b[q]) * rinv % p
            assert value(want) < 2 * p


@pytest.mark.parametrize("curve", ["k1", "r1"])
@pytest.mark.parametrize("spec", gen_fp29_asm.SUB_FUNCS, ids=[f[1] for f in gen_fp29_asm.SUB_FUNCS])
def test_sub_variants_match_product_then_subtract(curve, spec):
    """The *_sub blocks: product and subtraction in one REDC, then f29_fold,
    give the limbs of the product followed by a subtract-and-reduce pass with
    the same multiple of p (tests/test_fp29_model.py's F.mul(a, b, subs)),
    for operands and norm subtrahends at the top of their ranges; mul2 (a b + c d,
    one REDC) gives the limbs of F.mul2."""
    import test_fp29_model as model

    kinds, name, sub_spec, _ = spec
    with open(HDR) as f:
        funcs = parse_header(f.read())
    lines, ops = funcs["f29a_%s_%s" % (name, curve)]
    F = model.FIELDS[2 if curve == "k1" else 3]
    p = F.p
    rng = random.Random(hash((curve, name)) & 0xffff)

    def norm(top=False):  # a norm value (< 2p) in normalised limbs; top: 2p - 1
        v = 2 * p - 1 if top else rng.randrange(2 * p)
        return [(v >> (29 * i)) & M29 for i in range(8)] + [v >> 232]

    for it in range(40):
        edge = it < 2  # every operand and subtrahend at 2p - 1
        a = {0: norm(edge), 1: norm(edge)}
        b = {0: norm(edge), 1: norm(edge)}
        for q in range(len(kinds)):
            if kinds[q] == "sqr":
                b[q] = a[q]
        subs = {"c0": norm(edge), "d0": norm(edge)} if kinds[0] == "mul2" else {}
        for q, sp in enumerate(sub_spec):
            for j, sk in enumerate(sp):
                if sk == "e":
                    subs["s%d%d" % (q, j)] = norm(edge)
        got = emulate(lines, ops, a, b, subs)
        want = []
        for q in range(len(kinds)):
            if kinds[q] == "mul2":
                want.append(F.mul2(a[q], b[q], subs["c0"], subs["d0"]))
                continue
            if sub_spec[q] and sub_spec[q][0] == "o":
                ss = [want[0]] * len(sub_spec[q])
            else:
                ss = [subs["s%d%d" % (q, j)] for j in range(len(sub_spec[q]))]
            want.append(F.mul(a[q], b[q], tuple(ss)))
        for q in range(len(kinds)):
            if sub_spec[q]:
                g = F.fold(got[q][:8] + [0], got[q][8])
            else:
                g = got[q]
            assert g == want[q], (q, g, want[q])
