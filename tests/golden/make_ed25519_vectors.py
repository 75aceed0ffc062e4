#!/usr/bin/env python3
"""Generate tests/golden/ed25519_vectors.json — the committed Ed25519 fixture.

Run from the repo root:  python3 tests/golden/make_ed25519_vectors.py

Expected statuses come from the pure-Python restatement of i2p 0.2.0
(`oracle/i2p_ed25519.py`). Every vector also records OpenSSL 3's verdict
(`tests/golden/openssl_ed25519.py`, an independent RFC 8032 implementation);
categories where RFC 8032 and i2p 0.2.0 are known to agree are asserted to
agree here, so the restatement is pinned on them.

Categories follow SURVEY.md §8(d) C2's corruption catalogue plus the
reference tests' structural cases (`CryptoUtilsTest.kt:233-286`: round trip,
`sig[0]++` rejects, empty input throws) and Corda's fixed test keys
(`entropyToKeyPair(10..110)`, `test-utils/.../TestConstants.kt:27-69`).
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, HERE)

import i2p_ed25519 as ed  # noqa: E402
import openssl_ed25519 as ossl  # noqa: E402

P, L = ed.P, ed.L
rng = random.Random(0xC0DA0001)
vectors = []

# categories where RFC 8032 (OpenSSL) and i2p 0.2.0 must agree
AGREE = {"valid", "fixed_key", "r_bitflip", "s_bitflip", "msg_bitflip", "wrong_key",
         "sig0_increment", "long_msg", "random_sig"}


def add(cat, pub, sig, msg, note=""):
    st = ed.verify_status(pub, sig, msg)
    o = ossl.verify(pub, sig, msg) if (len(pub) == 32 and len(sig) and len(msg)) else None
    if cat in AGREE:
        assert o == (st == ed.OK), (cat, note, st, o)
    vectors.append({"cat": cat, "pub": pub.hex(), "sig": sig.hex(), "msg": msg.hex(),
                    "status": st, "openssl": o, "note": note})
    return st


def seed(i):
    return hashlib.sha256(b"corda-amd-golden-seed" + i.to_bytes(8, "little")).digest()


def txid(i):
    return hashlib.sha256(b"corda-amd-golden-tx" + i.to_bytes(8, "little")).digest()


def sign_both(sd, msg):
    pub, sig = ed.sign(sd, msg)
    assert sig == ossl.sign(sd, msg) and pub == ossl.keypair(sd)
    return pub, sig


# 1. valid (32-byte tx ids), signatures cross-checked bit-for-bit against OpenSSL
for i in range(64):
    m = txid(i)
    pub, sig = sign_both(seed(i), m)
    add("valid", pub, sig, m)

# 2. Corda's fixed test keys: entropyToKeyPair(10..110)
for ent in (10, 20, 30, 40, 50, 60, 70, 80, 90, 100, 110):
    m = txid(1000 + ent)
    pub, sig = sign_both(ed.entropy_seed(ent), m)
    add("fixed_key", pub, sig, m, note="entropy=%d" % ent)

# 3. structural corruption (reference: sig[0]++ must fail)
for i in range(16):
    m = txid(2000 + i)
    pub, sig = sign_both(seed(2000 + i), m)
    s = bytearray(sig)
    s[0] = (s[0] + 1) & 0xFF
    add("sig0_increment", pub, bytes(s), m)
    s = bytearray(sig)
    bit = rng.randrange(256)
    s[bit // 8] ^= 1 << (bit % 8)
    add("r_bitflip", pub, bytes(s), m, note="bit=%d" % bit)
    s = bytearray(sig)
    bit = 256 + rng.randrange(253)
    s[bit // 8] ^= 1 << (bit % 8)
    add("s_bitflip", pub, bytes(s), m, note="bit=%d" % (bit - 256))
    mm = bytearray(m)
    bit = rng.randrange(256)
    mm[bit // 8] ^= 1 << (bit % 8)
    add("msg_bitflip", pub, sig, bytes(mm), note="bit=%d" % bit)
    pub2, _ = sign_both(seed(3000 + i), m)
    add("wrong_key", pub2, sig, m)

# 4. S + kL (malleability; i2p has no S < L check) incl. slide() carry drop
for i in range(24):
    m = txid(4000 + i)
    pub, sig = sign_both(seed(4000 + i), m)
    S = int.from_bytes(sig[32:], "little")
    kmax = (2**256 - 1 - S) // L
    for k in sorted(set([1, 2, kmax // 2, kmax - 1, kmax] + [rng.randrange(1, kmax + 1) for _ in range(2)])):
        if k < 1:
            continue
        S2 = S + k * L
        sb = S2.to_bytes(32, "little")
        overflow = ed.slide_value(sb) != S2
        add("s_plus_kL", pub, sig[:32] + sb, m,
            note="k=%d bit255=%d slide_overflow=%d" % (k, S2 >> 255, int(overflow)))

# 5. extreme S values (slide overflow behaviour at the top of the range)
for i, S2 in enumerate([2**256 - 1, 2**255, 2**255 + 2**251, 2**256 - 2**250, L, 0, 1, L - 1,
                        2**253 - 1, 2**255 - 1]):
    m = txid(5000 + i)
    pub, sig = sign_both(seed(5000 + i), m)
    add("s_extreme", pub, sig[:32] + S2.to_bytes(32, "little"), m, note="S=%x" % S2)

# 6. non-canonical / special public keys
def enc_y(y, sign):
    b = bytearray((y % 2**255).to_bytes(32, "little"))
    b[31] |= sign << 7
    return bytes(b)


for y in range(0, 19):
    for sign in (0, 1):
        for noncanon in (False, True):
            yy = y + P if noncanon else y
            if yy >= 2**255:
                continue
            pub = enc_y(yy, sign)
            m = txid(6000 + y * 4 + sign * 2 + noncanon)
            A = ed.decode_i2p(pub)
            cat = "key_small_y" if not noncanon else "key_noncanonical_y"
            if A is None:
                add(cat, pub, os.urandom(0) + bytes(rng.getrandbits(8) for _ in range(64)), m, note="off-curve y=%d" % y)
                continue
            # accept-by-construction attempts for small-order keys: R = [S]B - [h]A
            S = rng.randrange(L)
            SB = ed.scalar_mult(S)
            made = False
            for kk in range(8):
                R = ed.encode(ed.pt_add(SB, ed.pt_neg(ed.scalar_mult(kk, A))))
                h = int.from_bytes(hashlib.sha512(R + ed.encode(A) + m).digest(), "little") % L
                if ed.encode(ed.scalar_mult(h, A)) == ed.encode(ed.scalar_mult(kk, A)):
                    add(cat, pub, R + S.to_bytes(32, "little"), m, note="y=%d sign=%d constructed" % (y, sign))
                    made = True
                    break
            if not made:
                add(cat, pub, bytes(rng.getrandbits(8) for _ in range(64)), m, note="y=%d sign=%d random-sig" % (y, sign))

# identity key with sign bit set (x = 0, bit 255 = 1): R = [S]B verifies for any message
for i in range(4):
    S = rng.randrange(L)
    m = txid(7000 + i)
    add("key_identity_signbit", enc_y(1, 1), ed.encode(ed.scalar_mult(S)) + S.to_bytes(32, "little"), m)
    add("key_identity_signbit", enc_y(1, 1), ed.encode(ed.scalar_mult(S)) + S.to_bytes(32, "little"), m[:31] + bytes([m[31] ^ 1]),
        note="any message accepted")

# 7. small-order and mixed-order keys (cofactorless equation)
torsion = [ed.decode_i2p(e) for e in ed.small_order_points()]
for ti, T in enumerate(torsion):
    sd = seed(8000 + ti)
    _, a, prefix = ed.seed_to_keypair(sd)
    Amixed = ed.pt_add(ed.scalar_mult(a), T)
    apub = ed.encode(Amixed)
    got = set()
    for j in range(40):
        m = txid(8100 + ti * 64 + j)
        r = int.from_bytes(hashlib.sha512(prefix + m).digest(), "little") % L
        R = ed.encode(ed.scalar_mult(r))
        h = int.from_bytes(hashlib.sha512(R + apub + m).digest(), "little") % L
        S = (r + h * a) % L
        st = ed.verify_status(apub, R + S.to_bytes(32, "little"), m)
        if st in got and j > 3:
            continue
        got.add(st)
        add("key_mixed_order", apub, R + S.to_bytes(32, "little"), m, note="torsion=%d" % ti)
    add("key_small_order", ed.encode(T), bytes(rng.getrandbits(8) for _ in range(64)), txid(8900 + ti))

# 8. non-canonical R encodings (y + p): never equal to the canonical encode(R')
for i in range(8):
    m = txid(9000 + i)
    pub, sig = sign_both(seed(9000 + i), m)
    y = rng.randrange(0, 19)
    add("r_noncanonical", pub, enc_y(y + P, rng.randrange(2)) + sig[32:], m)
# R = identity with sign bit (x = 0): canonical encode never sets it
for i in range(4):
    S = rng.randrange(L)
    m = txid(9100 + i)
    pub, sig = sign_both(seed(9100 + i), m)
    add("r_identity_signbit", pub, enc_y(1, 1) + sig[32:], m)

# 9. lengths / empties (Crypto.doVerify require checks, EdDSAEngine length check)
m = txid(9500)
pub, sig = sign_both(seed(9500), m)
add("sig_len", pub, sig[:63], m, note="63 bytes")
add("sig_len", pub, sig + b"\x00", m, note="65 bytes")
add("empty", pub, b"", m, note="empty signature")
add("empty", pub, sig, b"", note="empty clear data")
add("key_len", pub[:31], sig, m, note="31-byte key")
add("key_len", pub[:31], b"", m, note="31-byte key and empty signature: key decode first")
add("empty", enc_y(2, 0) if ed.decode_i2p(enc_y(2, 0)) is None else enc_y(3, 0), b"", m,
    note="off-curve key and empty signature: key decode first")
add("empty", pub, sig[:10], b"", note="empty clear data beats a short signature")

# 10. longer / odd-length messages (multi-block SHA-512)
for i, ln in enumerate([1, 31, 33, 64, 111, 112, 127, 128, 200, 1000]):
    msg = bytes(rng.getrandbits(8) for _ in range(ln))
    pub, sig = sign_both(seed(9600 + i), msg)
    add("long_msg", pub, sig, msg, note="len=%d" % ln)

# 11. random garbage signatures on valid keys
for i in range(16):
    m = txid(9700 + i)
    pub, _ = sign_both(seed(9700 + i), m)
    add("random_sig", pub, bytes(rng.getrandbits(8) for _ in range(64)), m)

out = os.path.join(HERE, "ed25519_vectors.json")
with open(out, "w") as f:
    json.dump({"generator": "tests/golden/make_ed25519_vectors.py",
               "oracle": "oracle/i2p_ed25519.py (i2p eddsa 0.2.0 restatement)",
               "independent": "OpenSSL %s libcrypto (RFC 8032)" % "3",
               "vectors": vectors}, f, indent=0)
from collections import Counter
print(len(vectors), "vectors ->", out)
print(Counter((v["cat"], v["status"]) for v in vectors))
