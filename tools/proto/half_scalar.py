"""Prototype (dev tool, not a test oracle): Ed25519 cofactorless verification
with half-size scalars (Pornin 2020 idea, exact for torsion): find (c0, c1)
with c0 = c1*h (mod 8L), |c0|,|c1| ~ 2^128, c1 odd; then
  encode([S]B - [h]A) == R  <=>  R canonical & on curve & [c1 S]B - [c0]A - [c1]R == O.
Checks the identity against the i2p restatement on the golden vectors."""
import json, os, sys, random
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import hashlib
import i2p_ed25519 as ed

L, P = ed.L, ed.P
M = 8 * L


def glv_basis(h, m=M):
    """Extended Euclid on (m, h); GLV-style short basis."""
    r = [m, h]
    t = [0, 1]
    import math
    s = math.isqrt(m)
    while r[-1] >= s:
        q = r[-2] // r[-1]
        r.append(r[-2] - q * r[-1])
        t.append(t[-2] - q * t[-1])
    # r[-1] < sqrt(m) <= r[-2]
    l = len(r) - 2
    v1 = (r[l + 1], t[l + 1])
    q = r[l] // r[l + 1]
    r2 = r[l] - q * r[l + 1]
    t2 = t[l] - q * t[l + 1]
    cand = [(r[l], t[l]), (r2, t2)]
    v2 = min(cand, key=lambda v: v[0] ** 2 + v[1] ** 2)
    return v1, v2, len(r) - 2


def pick(h):
    v1, v2, steps = glv_basis(h)
    cands = [v1, v2, (v1[0] + v2[0], v1[1] + v2[1]), (v1[0] - v2[0], v1[1] - v2[1])]
    odd = [v for v in cands if v[1] % 2 != 0]
    best = min(odd, key=lambda v: max(abs(v[0]), abs(v[1])))
    assert (best[0] - best[1] * h) % M == 0
    return best, steps


def decode_strict(b):
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)
    if y >= P:
        return None
    pt = ed.decode_i2p(b)
    if pt is None:
        return None
    if pt[0] == 0 and (b[31] >> 7):
        return None
    return pt


def verify_half(pub, sig, msg):
    A = ed.decode_i2p(pub)
    if A is None:
        return ed.BAD_KEY
    if len(sig) == 0 or len(msg) == 0:
        return ed.EMPTY
    if len(sig) != 64:
        return ed.MALFORMED_SIG
    R = decode_strict(sig[:32])
    if R is None:
        return ed.BAD_SIG
    h = int.from_bytes(hashlib.sha512(sig[:32] + ed.encode(A) + msg).digest(), "little") % L
    S = ed.slide_value(sig[32:])  # S or S - 2^256
    (c0, c1), _ = pick(h)
    e = (c1 * S) % L
    Pt = ed.scalar_mult(e)
    nA = ed.scalar_mult(abs(c0), A)
    if c0 > 0:
        nA = ed.pt_neg(nA)
    cR = ed.scalar_mult(abs(c1), R)
    if c1 > 0:
        cR = ed.pt_neg(cR)
    Q = ed.pt_add(ed.pt_add(Pt, nA), cR)
    X, Y, Z, _ = Q
    return ed.OK if X % P == 0 and (Y - Z) % P == 0 else ed.BAD_SIG


if __name__ == "__main__":
    V = json.load(open(os.path.join(ROOT, "tests", "golden", "ed25519_vectors.json")))["vectors"]
    bad = 0
    for v in V:
        p, s, m = (bytes.fromhex(v[k]) for k in ("pub", "sig", "msg"))
        if verify_half(p, s, m) != v["status"]:
            bad += 1
            print("MISMATCH", v["cat"], v["note"])
    print("golden mismatches:", bad, "of", len(V))
    rng = random.Random(1)
    mx, st = 0, []
    for _ in range(20000):
        h = rng.randrange(L)
        (c0, c1), steps = pick(h)
        mx = max(mx, abs(c0).bit_length(), abs(c1).bit_length())
        st.append(steps)
    print("max bits of |c0|,|c1|:", mx, " euclid steps avg/max:", sum(st) / len(st), max(st))


def simple_pick(h, m=M):
    """GPU rule: Euclid until r_cur < sqrt(m); take (r_cur, t_cur) if t_cur odd, else one more step."""
    import math
    s = math.isqrt(m) + 1
    rp, rc, tp, tc = m, h, 0, 1
    steps = 0
    while rc >= s:
        q = rp // rc
        rp, rc = rc, rp - q * rc
        tp, tc = tc, tp - q * tc
        steps += 1
    if tc % 2:
        return (rc, tc), steps
    q = rp // rc if rc else 0
    return (rp - q * rc, tp - q * tc), steps + 1


if __name__ == "__main__":
    from collections import Counter
    rng = random.Random(2)
    cnt = Counter()
    for _ in range(100000):
        h = rng.randrange(L)
        (c0, c1), _ = simple_pick(h)
        assert (c0 - c1 * h) % M == 0 and c1 % 2
        cnt[max(abs(c0).bit_length(), abs(c1).bit_length())] += 1
    print(sorted(cnt.items()))


def pick2(h, m=M):
    import math
    s = math.isqrt(m) + 1
    rp, rc, tp, tc = m, h, 0, 1
    while rc >= s:
        q = rp // rc
        rp, rc = rc, rp - q * rc
        tp, tc = tc, tp - q * tc
    q = rp // rc if rc else 0
    v1, v3 = (rc, tc), (rp - q * rc, tp - q * tc)
    cands = [v1, v3, (v1[0] + v3[0], v1[1] + v3[1]), (v1[0] - v3[0], v1[1] - v3[1])]
    odd = [v for v in cands if v[1] % 2]
    return min(odd, key=lambda v: max(abs(v[0]).bit_length(), abs(v[1]).bit_length()))


if __name__ == "__main__":
    rng = random.Random(3)
    cnt = Counter()
    for _ in range(100000):
        h = rng.randrange(L)
        c0, c1 = pick2(h)
        assert (c0 - c1 * h) % M == 0 and c1 % 2
        cnt[max(abs(c0).bit_length(), abs(c1).bit_length())] += 1
    print("pick2", sorted(cnt.items()))
