"""Prototype (dev tool, not a test oracle) of the Ed25519 prep's lattice
reduction as Lehmer rounds (Knuth TAOCP 4.5.2 Algorithm L) over 52-bit
leading parts held exactly in doubles, with a threshold stop so that the
multiprecision remainder never drops below isqrt(8L)+1 inside a round. The
quotient sequence is Euclid's exactly, so the hand-off state and the chosen
(c0, c1) must equal the plain Euclid's (half_scalar.simple_pick's sequence).
Python floats are IEEE doubles with correctly rounded division, as on the GPU.

    python tools/proto/lehmer.py [N]
"""
import math
import random
import sys

L = 2**252 + 27742317777372353535851937790883648493
M = 8 * L
T = math.isqrt(M) + 1
MASK = (1 << 256) - 1


def euclid_state(h):
    """plain Euclid until the current remainder drops below T"""
    rp, rc, tp, tc = M, h, 0, 1
    steps = 0
    while rc >= T:
        q = rp // rc
        rp, rc = rc, rp - q * rc
        tp, tc = tc, tp - q * tc
        steps += 1
    return rp, rc, tp, tc, steps


def lehmer_state(h, stats):
    rp, rc, tp, tc = M, h, 0, 1  # tp, tc kept mod 2^256 as on the GPU
    tc &= MASK
    rounds = 0
    while True:
        s = max(rp.bit_length() - 52, 0)
        uh, vh = float(rp >> s), float(rc >> s)
        th = float((T >> s) + 1)
        A, B, C, D = 1.0, 0.0, 0.0, 1.0
        n = 0
        while True:
            d1, d2 = vh + C, vh + D
            if d1 <= 0 or d2 <= 0:
                break
            n1 = uh + A
            q = math.floor(n1 / d1)
            r1 = n1 - q * d1  # exact (fma on the GPU)
            q -= r1 < 0
            q += r1 >= d1
            r2 = (uh + B) - q * d2
            if r2 < 0 or r2 >= d2:
                break
            nC, nD = A - q * C, B - q * D
            nv = uh - q * vh
            if nv - max(abs(nC), abs(nD)) < th or max(abs(nC), abs(nD)) >= 2**30:
                break
            A, B, C, D = C, D, nC, nD
            uh, vh = vh, nv
            n += 1
        stats["small"] = stats.get("small", 0) + n
        stats["max_small"] = max(stats.get("max_small", 0), n)
        if n == 0:
            break
        rounds += 1
        a, b, c, d = int(A), int(B), int(C), int(D)
        assert max(abs(a), abs(b), abs(c), abs(d)) < 2**30
        rp, rc = a * rp + b * rc, c * rp + d * rc
        assert 0 <= rc < rp < 2**256 and rc >= T
        tp, tc = (a * tp + b * tc) & MASK, (c * tp + d * tc) & MASK
    stats["rounds"] = stats.get("rounds", 0) + rounds
    stats["max_rounds"] = max(stats.get("max_rounds", 0), rounds)
    fin = 0
    while rc >= T:
        q = rp // rc
        rp, rc = rc, rp - q * rc
        tp, tc = tc, (tp - q * tc) & MASK
        fin += 1
    stats["finish"] = stats.get("finish", 0) + fin
    stats["max_finish"] = max(stats.get("max_finish", 0), fin)
    sg = lambda x: x - (1 << 256) if x >> 255 else x
    return rp, rc, sg(tp), sg(tc)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    rng = random.Random(5)
    stats, esteps = {}, 0
    hs = [0, 1, 2, L - 1, T, T - 1, T + 1, M // 3 % L] + [rng.randrange(L) for _ in range(n)]
    for h in hs:
        *ref, st = euclid_state(h)
        esteps += st
        got = lehmer_state(h, stats)
        assert tuple(got) == tuple(ref), (h, got, ref)
    k = len(hs)
    print(f"{k} h values: Lehmer hand-off == Euclid's; Euclid steps avg {esteps / k:.1f}; "
          f"rounds avg {stats['rounds'] / k:.2f} max {stats['max_rounds']}; small steps avg {stats['small'] / k:.1f} "
          f"max/round {stats['max_small']}; exact finish steps avg {stats['finish'] / k:.2f} max {stats['max_finish']}")


if __name__ == "__main__":
    main()
