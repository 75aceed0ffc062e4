"""Limb-level model of fp29.hpp (kernel K2's base-field arithmetic) and of
ecdsa.hip's point formulas, run on the CPU.

Each operation mirrors the device code step for step on Python ints and
asserts what the device relies on: every 64-bit column accumulator of
f29_mul / f29_sqr stays below 2^64, every 32-bit limb below 2^32, every
Montgomery column clears its low 29 bits, and every result is the right
residue inside its documented value bound (fp29.hpp header). The point
formulas (jdbl for a = -3 and a = 0, jadd, jmadd, including their exceptional
branches) run on random Jacobian representatives pushed to the top of the
allowed range and are compared with the BouncyCastle restatement's affine
arithmetic (oracle/bc_ecdsa.py, the checker). The constants come from
tools/gen_fp29_consts.py; the committed header must match its output.
"""
import os
import random
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bc_ecdsa as ec  # noqa: E402  (oracle: checker only)
import gen_fp29_consts as gen  # noqa: E402

U32, U64 = 1 << 32, 1 << 64
M29 = (1 << 29) - 1
R = 1 << 261


class Fp29:
    def __init__(self, p, kred):
        self.p, self.kred = p, kred
        self.m = gen.limbs29(p)
        self.minv = gen.minv29(p)
        self.s2p = gen.sub2p(p)
        self.skp = {2: self.s2p, 4: gen.subkp(p, 4), 6: gen.subkp(p, 6)}
        self.r2 = gen.limbs29(R * R % p)
        self.one = gen.limbs29(R % p)

    @staticmethod
    def val(a):
        return sum(v << (29 * i) for i, v in enumerate(a))

    def mul(self, a, b, subs=()):
        """f29_mul; with subs, the fp29_asm.hpp *_sub variants: output column
        9 + i also accumulates limb i of kp - sum subs (k = 4, or 6 for three),
        the top limb wraps mod 2^32, then f29_fold (fp29.hpp)."""
        assert all(0 <= x < U32 for x in a + b)
        va, vb = self.val(a), self.val(b)
        assert va * vb < R * self.p, "Montgomery input bound a b < R p"
        if subs:
            skp = self.skp[4 if len(subs) <= 2 else 6]
            for sb in subs:
                assert self.val(sb) < 2 * self.p and all(x < (1 << 29) + (1 << 15) for x in sb[:8])
            xs = [skp[i] - sum(sb[i] for sb in subs) for i in range(9)]
            assert all(0 <= x < U32 for x in xs[:8])
        q, t, acc = [0] * 9, [0] * 9, 0
        for k in range(17):
            acc += sum(a[j] * b[k - j] for j in range(max(0, k - 8), min(k, 8) + 1))
            acc += sum(q[j] * self.m[k - j] for j in range(max(0, k - 8), min(k, 9)))
            if k < 9:
                q[k] = ((acc % U32) * self.minv % U32) & M29
                acc += q[k] * self.m[0]
                assert acc & M29 == 0
            else:
                if subs:
                    acc += xs[k - 9]
                t[k - 9] = acc & M29
            assert acc < U64, "column %d overflows" % k
            acc >>= 29
        if subs:
            top = (acc + xs[8]) % U32
            assert top == acc + xs[8], "the folded top stays below 2^32 as a value"
            out = self.fold(t[:8] + [0], top)
            want = (va * vb * pow(R, -1, self.p) - sum(self.val(sb) for sb in subs)) % self.p
            assert self.val(out) % self.p == want
            return out
        t[8] = acc
        assert t[8] < U32
        assert self.val(t) % self.p == va * vb * pow(R, -1, self.p) % self.p
        assert self.val(t) < 2 * self.p
        return t

    def sqr(self, a):
        assert all(2 * x < U32 for x in a)  # the doubled operand a2[j] = a[j] << 1
        return self.mul(a, a)               # same column sums as the symmetric schedule

    @staticmethod
    def add(a, b):
        r = [x + y for x, y in zip(a, b)]
        assert all(x < U32 for x in r)
        return r

    def sub(self, a, b):
        assert self.val(b) <= 2 * self.p
        r, c = [0] * 9, 0
        for i in range(8):
            t = a[i] + self.s2p[i] - b[i] + c
            assert 0 <= t < U32
            r[i], c = t & M29, t >> 29
        r[8] = a[8] + self.s2p[8] - b[8] + c
        assert 0 <= r[8] < U32
        assert self.val(r) == self.val(a) + 2 * self.p - self.val(b)
        return r

    def fold(self, r, top):
        """fp29.hpp f29_fold: limbs 0..7 normalised, top = bits >= 2^232."""
        assert all(0 <= x <= M29 for x in r[:8]) and 0 <= top < U32
        v_in = self.val(r[:8] + [top])
        assert v_in < 1 << 260
        r = list(r)
        q = top >> 24
        r[8] = top & 0xFFFFFF
        if self.kred == 1:
            r[0] += q * 977
            r[1] += q << 3
        else:
            r[0] += q
            r[3] -= q << 9
            r[6] -= q << 18
            r[7] += q << 21
            for i in range(3, 8):
                assert -(1 << 31) <= r[i] < 1 << 31
                cs = r[i] >> 29          # arithmetic shift, as (int32_t) >> 29
                r[i] &= M29
                r[i + 1] += cs
        assert all(0 <= x < U32 for x in r)
        assert all(x < (1 << 29) + (1 << 15) for x in r[:8])
        assert self.val(r) % self.p == v_in % self.p and self.val(r) < 2 * self.p
        return r

    def red(self, a):
        assert all(0 <= x < U32 for x in a) and self.val(a) < 1 << 260
        r, c = [0] * 9, 0
        for i in range(8):
            t = a[i] + c
            assert t < U32
            r[i], c = t & M29, t >> 29
        top = a[8] + c
        assert top < U32
        return self.fold(r, top)

    def subs_red(self, a, *bs):
        """f29_sub_red / f29_sub2_red / f29_sub3_red: red(a + 2k p - sum bs) in one pass."""
        k = 2 * len(bs)
        s = self.skp[k]
        for b in bs:
            assert self.val(b) <= 2 * self.p and all(x < (1 << 29) + (1 << 15) for x in b)
        r, c = [0] * 9, 0
        for i in range(8):
            t = a[i] + s[i] - sum(b[i] for b in bs) + c
            assert 0 <= t < U32, "limb %d out of range" % i
            r[i], c = t & M29, t >> 29
        top = a[8] + s[8] - sum(b[8] for b in bs) + c
        assert 0 <= top < U32
        out = self.fold(r, top)
        assert self.val(out) % self.p == (self.val(a) - sum(self.val(b) for b in bs)) % self.p
        return out

    def mulk_red(self, a, k):
        """f29_mulk_red: red(k a) in one pass, a norm."""
        r, c = [0] * 9, 0
        for i in range(8):
            t = a[i] * k + c
            assert t < U32
            r[i], c = t & M29, t >> 29
        top = a[8] * k + c
        assert top < U32
        return self.fold(r, top)

    def mulk_carry(self, a, k):
        """f29_mulk_carry: k a with one carry pass, no fold (limbs 0..7 normalised,
        the top limb keeps the rest); a a REDC output (value < 1.5p), k = 3."""
        assert self.val(a) < 3 * self.p // 2
        r, c = [0] * 9, 0
        for i in range(8):
            t = a[i] * k + c
            assert t < U32
            r[i], c = t & M29, t >> 29
        r[8] = a[8] * k + c
        assert r[8] < U32 and self.val(r) == k * self.val(a)
        return r

    def neg2_norm(self, a):
        """fp29.hpp f29_neg2_norm: 4p - 2a for a norm a, one carry pass."""
        s4 = self.skp[4]
        assert self.val(a) < 2 * self.p and all(x < (1 << 29) + (1 << 15) for x in a[:8])
        r, c = [0] * 9, 0
        for i in range(8):
            t = s4[i] - 2 * a[i] + c
            assert 0 <= t < U32
            r[i], c = t & M29, t >> 29
        r[8] = s4[8] - 2 * a[8] + c
        assert 0 <= r[8] < U32 and self.val(r) == 4 * self.p - 2 * self.val(a)
        return r

    def mul2(self, a, b, c, d):
        """fp29_asm.hpp mul2: a b + c d in the same 64-bit columns, one REDC."""
        assert all(0 <= x < U32 for x in a + b + c + d)
        va, vb, vc, vd = (self.val(x) for x in (a, b, c, d))
        assert va * vb + vc * vd < R * self.p, "Montgomery input bound"
        q, t, acc = [0] * 9, [0] * 9, 0
        for k in range(17):
            rng = range(max(0, k - 8), min(k, 8) + 1)
            acc += sum(a[j] * b[k - j] + c[j] * d[k - j] for j in rng)
            acc += sum(q[j] * self.m[k - j] for j in range(max(0, k - 8), min(k, 9)))
            if k < 9:
                q[k] = ((acc % U32) * self.minv % U32) & M29
                acc += q[k] * self.m[0]
                assert acc & M29 == 0
            else:
                t[k - 9] = acc & M29
            assert acc < U64, "column %d overflows" % k
            acc >>= 29
        t[8] = acc
        assert t[8] < U32
        assert self.val(t) % self.p == (va * vb + vc * vd) * pow(R, -1, self.p) % self.p
        assert self.val(t) < 2 * self.p
        return t

    def canon(self, a):
        t = self.red(a)
        c = 0
        for i in range(8):
            s = t[i] + c
            t[i], c = s & M29, s >> 29
        t[8] += c
        d, br = [0] * 9, 0
        for i in range(9):
            s = (t[i] - self.m[i] - br) % U32
            d[i], br = s & M29, s >> 31
        r = d if br == 0 else t
        assert self.val(r) == self.val(a) % self.p
        return r

    def iszero(self, a):
        return not any(self.canon(a))

    def iszero_norm(self, a):
        """fp29.hpp f29_iszero_norm: one carry pass, compare with 0 and p (a norm)."""
        assert self.val(a) < 2 * self.p and all(0 <= x < U32 for x in a)
        c, limbs = 0, []
        for i in range(8):
            s = a[i] + c
            assert s < U32
            limbs.append(s & M29)
            c = s >> 29
        limbs.append(a[8] + c)
        r = limbs == [0] * 9 or limbs == list(self.m)
        assert r == self.iszero(a)
        return r

    def neg(self, a):
        return self.sub([0] * 9, a)

    def sub_loose(self, a, b):
        """fp29.hpp f29_sub_loose: a + 4p - b limb by limb, no carry."""
        s4 = self.skp[4]
        assert self.val(b) <= 2 * self.p and all(x < (1 << 29) + (1 << 15) for x in b[:8])
        r = [a[i] + s4[i] - b[i] for i in range(9)]
        assert all(0 <= x < U32 for x in r)
        assert self.val(r) == self.val(a) + 4 * self.p - self.val(b)
        return r

    def cneg_loose(self, a):
        """fp29.hpp f29_cneg_loose (negating case): 4p - a limb by limb, no carry."""
        s4 = self.skp[4]
        assert self.val(a) < 2 * self.p and all(x < (1 << 29) + (1 << 15) for x in a[:8])
        r = [s4[i] - a[i] for i in range(9)]
        assert all(0 <= x < U32 for x in r)
        assert self.val(r) == 4 * self.p - self.val(a)
        return r

    def to_mont(self, x):
        return self.mul(gen.limbs29(x), self.r2)

    def from_mont(self, a):
        return self.val(self.canon(self.mul(a, [1] + [0] * 8)))


FIELDS = {2: Fp29(gen.P_K1, 1), 3: Fp29(gen.P_R1, 2)}
AM3 = {2: False, 3: True}


# ---- ecdsa.hip's point formulas, op for op -----------------------------------
def jdbl(F, am3, P):
    if P is None:
        return None
    X, Y, Z = P
    if am3:
        delta, gamma = F.sqr(Z), F.sqr(Y)
        t, u = F.sub(X, delta), F.add(X, delta)
        x4 = F.add(F.add(X, X), F.add(X, X))
        b4, a3 = F.mul(x4, gamma), F.mul(t, u)      # 4 beta = (4 X) gamma: no mulk_red pass
        a3 = F.mulk_carry(a3, 3)                    # alpha < 4.5p, not folded
        x3 = F.mul(a3, a3, (b4, b4))                # X3 = alpha^2 - 8 beta, folded into the REDC
        z3 = F.mul(F.add(Y, Y), Z)                  # Z3 = 2 Y Z as one product
        u = F.sub_loose(b4, x3)
        t = F.sqr(F.add(gamma, gamma))
        y3 = F.mul(a3, u, (t, t))                   # Y3 = alpha (4 beta - X3) - 8 gamma^2
    else:
        A, B = F.sqr(X), F.sqr(Y)
        x4 = F.add(F.add(X, X), F.add(X, X))
        C, D = F.sqr(B), F.mul(x4, B)           # D = 2((X + B)^2 - A - C) = 4 X B, one product
        E = F.mulk_carry(A, 3)                  # E = 3 A, not folded
        t = F.add(Y, Y)
        x3, z3 = F.mul(E, E, (D, D)), F.mul(t, Z)  # X3 = E^2 - 2 D folded into the REDC
        u = F.mulk_red(C, 4)
        y3 = F.mul(E, F.sub_loose(D, x3), (u, u))   # Y3 = E (D - X3) - 8 C
    return (x3, y3, z3)


def jadd(F, am3, P, Q):
    if P is None:
        return Q
    if Q is None:
        return P
    (X1, Y1, Z1), (X2, Y2, Z2) = P, Q
    z1z1, z2z2 = F.sqr(Z1), F.sqr(Z2)
    u1, u2 = F.mul(X1, z2z2), F.mul(X2, z1z1)
    s1 = F.mul(F.mul(Y1, Z2), z2z2)
    s2 = F.mul(F.mul(Y2, Z1), z1z1)
    h, rr = F.red(F.sub(u2, u1)), F.red(F.sub(s2, s1))
    if F.iszero(h):
        return jdbl(F, am3, P) if F.iszero(rr) else None
    i = F.sqr(F.add(h, h))
    j = F.mul(h, i)
    rr = F.add(rr, rr)
    v = F.mul(u1, i)
    x3 = F.red(F.sub(F.sub(F.sub(F.sqr(rr), j), v), v))
    y3 = F.mul(rr, F.sub(v, x3))
    t = F.mul(s1, j)
    y3 = F.red(F.sub(F.sub(y3, t), t))
    t = F.sub(F.sub(F.sqr(F.add(Z1, Z2)), z1z1), z2z2)
    return (x3, y3, F.mul(t, h))


def jmadd(F, am3, P, x2, y2):
    if P is None:
        return (x2, F.red(y2), list(F.one))
    X1, Y1, Z1 = P
    z1z1, t = F.sqr(Z1), F.mul(y2, Z1)
    h, rr = F.mul(x2, z1z1, (X1,)), F.mul(t, z1z1, (Y1,))  # H = U2 - X1, R = S2 - Y1 (+4p)
    if F.iszero_norm(h):
        return jdbl(F, am3, P) if F.iszero_norm(rr) else None
    rr = F.add(rr, rr)
    hh = F.sqr(h)
    i = F.add(hh, hh)
    i = F.add(i, i)
    j, v = F.mul(h, i), F.mul(X1, i)
    x3 = F.mul(rr, rr, (j, v, v))                   # X3 = r^2 - J - 2 V (+6p)
    y3 = F.mul2(rr, F.sub(v, x3), Y1, F.neg2_norm(j))  # Y3 = r (V - X3) + Y1 (4p - 2J), one REDC
    z3 = F.mul(F.add(Z1, Z1), h)                    # Z3 = 2 Z1 H
    return (x3, y3, z3)


def affine(F, P):
    if P is None:
        return None
    X, Y, Z = (F.from_mont(c) for c in P)
    zi = pow(Z, -1, F.p)
    return (X * zi * zi % F.p, Y * zi * zi * zi % F.p)


def high(F, x, rng):
    """Montgomery form of x as a norm value, pushed to [p, 2p) half the time."""
    v = F.val(F.canon(F.to_mont(x)))
    if rng.random() < 0.5 and v + F.p < 2 * F.p:
        v += F.p
    return gen.limbs29(v)


def jacobian(F, pt, rng):
    z = rng.randrange(1, F.p)
    x, y = pt
    return (high(F, x * z * z % F.p, rng), high(F, y * z * z * z % F.p, rng), high(F, z, rng))


def rand_point(c, rng):
    return ec._mul(c, rng.randrange(1, c.n), c.G)


def test_header_matches_generator():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_fp29_consts.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("scheme", [2, 3])
def test_field_ops_extremes(scheme):
    F = FIELDS[scheme]
    rng = random.Random(scheme)
    p = F.p
    edge = [0, 1, p - 1, p, p + 1, 2 * p - 1, (1 << 256) - 1 if (1 << 256) - 1 < 2 * p else 2 * p - 2]
    vals = edge + [rng.randrange(2 * p) for _ in range(200)]
    for a in vals:
        la = gen.limbs29(a)
        for b in rng.sample(vals, 4):
            lb = gen.limbs29(b)
            F.mul(la, lb)
            F.mul(F.add(la, la), F.add(lb, lb))           # 4p x 4p
            F.sub(la, lb)
            F.red(F.add(F.add(la, la), F.add(la, la)))    # 8p, limbs < 2^31
            m = F.mul(la, lb)                               # norm minuends / subtrahends
            F.subs_red(m, la)
            F.subs_red(m, la, lb)
            F.subs_red(m, la, lb, la)
            F.mulk_red(la, 4)
        F.sqr(F.add(la, la))
        assert F.val(F.canon(la)) == a % p
        assert F.from_mont(F.to_mont(a % p)) == a % p


@pytest.mark.parametrize("scheme", [2, 3])
def test_point_formulas_vs_affine(scheme):
    F, c, am3 = FIELDS[scheme], ec.CURVES[scheme], AM3[scheme]
    rng = random.Random(10 + scheme)
    for _ in range(25):
        P, Q = rand_point(c, rng), rand_point(c, rng)
        JP, JQ = jacobian(F, P, rng), jacobian(F, Q, rng)
        assert affine(F, jdbl(F, am3, JP)) == ec._add(c, P, P)
        assert affine(F, jadd(F, am3, JP, JQ)) == ec._add(c, P, Q)
        xq, yq = high(F, Q[0], rng), high(F, Q[1], rng)
        assert affine(F, jmadd(F, am3, JP, xq, yq)) == ec._add(c, P, Q)
        # chained: outputs feed further ops (the ladder's shape)
        S = jdbl(F, am3, jdbl(F, am3, jadd(F, am3, JP, JQ)))
        assert affine(F, jmadd(F, am3, S, xq, yq)) == ec._add(c, ec._mul(c, 4, ec._add(c, P, Q)), Q)


@pytest.mark.parametrize("scheme", [2, 3])
def test_exceptional_additions(scheme):
    F, c, am3 = FIELDS[scheme], ec.CURVES[scheme], AM3[scheme]
    rng = random.Random(20 + scheme)
    P = rand_point(c, rng)
    JP, JP2 = jacobian(F, P, rng), jacobian(F, P, rng)
    assert affine(F, jadd(F, am3, JP, JP2)) == ec._add(c, P, P)            # P + P -> doubling
    negP = (P[0], (-P[1]) % F.p)
    assert jadd(F, am3, JP, jacobian(F, negP, rng)) is None                 # P - P -> infinity
    assert affine(F, jmadd(F, am3, JP, high(F, P[0], rng), high(F, P[1], rng))) == ec._add(c, P, P)
    assert jmadd(F, am3, JP, high(F, P[0], rng), F.neg(high(F, P[1], rng))) is None


@pytest.mark.parametrize("scheme", [2, 3])
def test_iszero_norm_on_sub_red_outputs(scheme):
    """f29_iszero_norm agrees with the canonicalising test on every norm value
    a sub_red can produce near 0 and p, including non-normalised limbs 0, 1
    (fold outputs) and the two representatives 0 and p of zero."""
    F = FIELDS[scheme]
    rng = random.Random(30 + scheme)
    p = F.p
    vals = [0, 1, 2, p - 2, p - 1, p, p + 1, p + 2, 2 * p - 1] + [rng.randrange(2 * p) for _ in range(300)]
    hits = 0
    for a in vals:
        for b in [0, 1, p - 1, p, a % p, (a + 1) % p] + [rng.randrange(2 * p) for _ in range(6)]:
            m = F.mul(gen.limbs29(a), F.r2)             # a norm product output
            bb = F.mul(gen.limbs29(b), F.r2)
            h = F.subs_red(m, bb)                       # the addition's H = U2 - X1, as the kernel makes it
            hits += F.iszero_norm(h)
            F.iszero_norm(gen.limbs29(a))               # normalised limbs
    assert hits > 0
    # explicit non-normalised limbs: limb 0 carrying into limb 1 (fold excess)
    for v in (0, p):
        l = gen.limbs29(v)
        if l[1] > 0:
            l2 = list(l)
            l2[1] -= 1
            l2[0] += 1 << 29
            assert F.iszero_norm(l2)


@pytest.mark.parametrize("scheme", [2, 3])
def test_mixed_addition_with_loose_negated_y(scheme):
    """The ladder's table and fixed-base y, negated by f29_cneg_loose (4p - y,
    no carry), into jmadd: every product column stays < 2^64 (F.mul asserts it),
    the sum is P - Q, and the infinity branch returns a norm Y."""
    F, c, am3 = FIELDS[scheme], ec.CURVES[scheme], AM3[scheme]
    rng = random.Random(40 + scheme)
    for _ in range(25):
        P, Q = rand_point(c, rng), rand_point(c, rng)
        JP = jacobian(F, P, rng)
        xq, yq = high(F, Q[0], rng), high(F, Q[1], rng)
        negQ = (Q[0], (-Q[1]) % F.p)
        assert affine(F, jmadd(F, am3, JP, xq, F.cneg_loose(yq))) == ec._add(c, P, negQ)
        S = jmadd(F, am3, None, xq, F.cneg_loose(yq))     # accumulator at infinity
        assert F.val(S[1]) < 2 * F.p and affine(F, S) == negQ
        assert affine(F, jdbl(F, am3, S)) == ec._add(c, negQ, negQ)
    # extreme limbs: y = 0 (4p - 0) and y just below 2p
    for yv in (0, 2 * F.p - 1):
        y = gen.limbs29(yv)
        F.mul(F.cneg_loose(y), gen.limbs29(2 * F.p - 1))


def test_glv_split_bound():
    assert gen.check() <= 129


def max_columns(F, amax, bmax, sqr=False, xmax=0, cmax=None, dmax=None):
    """Upper bound of every 64-bit column value of f29_mul (P-256 special-form
    REDC terms, q_k < 2^29) from per-limb upper bounds of the operands, plus
    an added term < xmax in the output columns (the *_sub variants) and, for
    mul2, the second product c d in the same columns."""
    cols, carry = [], 0
    for k in range(17):
        s = carry
        for j in range(max(0, k - 8), min(k, 8) + 1):
            s += amax[j] * bmax[k - j]
            if cmax:
                s += cmax[j] * dmax[k - j]
        s += sum(M29 * c for c, lo, hi, off in ((1 << 9, 3, 11, 3), (1 << 18, 6, 14, 6), (F.m[7], 7, 15, 7),
                                                 (F.m[8], 8, 16, 8)) if lo <= k <= hi)
        if k < 9:
            s += M29  # the p == -1 term: column + (2^29 - 1) q... bounded by one more 2^29
        else:
            s += xmax
        cols.append(s)
        carry = s >> 29
    return cols


def test_alpha_products_worst_case_columns():
    """P-256 doubling with the unfolded alpha = 3 m (m a REDC output < 1.5p):
    alpha^2 and alpha (4 beta - X3) (a sub_loose operand) stay below 2^64 in
    every column for the worst limb of every operand, not just sampled ones."""
    F = FIELDS[3]
    norm = [(1 << 29) + (1 << 15)] * 2 + [1 << 29] * 6 + [1 << 25]
    alpha = [1 << 29] * 8 + [((9 * F.p) // 2 >> 232) + 1]
    loose = [norm[i] + F.skp[4][i] for i in range(9)]  # b4 + 4p - x3, b4 norm
    for a, b, sq, xm in ((alpha, alpha, True, U32), (alpha, loose, False, U32)):
        cols = max_columns(F, a, b, sq, xm)
        assert max(cols) < U64, [c.bit_length() for c in cols]
    assert (9 * F.p // 2) ** 2 < R * F.p and (9 * F.p // 2) * 6 * F.p < R * F.p
    # mixed addition's Y3 = r (V - X3) + Y1 (4p - 2J) as one REDC: r = 2R (limbs
    # of two norms), V - X3 and 4p - 2J carry-normalised (f29_sub, f29_neg2_norm)
    rr = [2 * x for x in norm]
    nrm = [1 << 29] * 8 + [((6 * F.p) >> 232) + 1]
    cols = max_columns(F, rr, nrm, False, 0, norm, nrm)
    assert max(cols) < U64, [c.bit_length() for c in cols]
    assert 4 * F.p * 4 * F.p + 2 * F.p * 4 * F.p < R * F.p
