#!/usr/bin/env python3
"""Generate tests/golden/ecdsa_vectors.json (secp256k1 = scheme 2, P-256 = 3).

Expected statuses: oracle/bc_ecdsa.py (BouncyCastle 1.57 restatement). Every
vector is also run through OpenSSL 3 ECDSA_verify; where BC and OpenSSL share
the rule (all categories here except the UNPINNED key encodings), agreement is
asserted: OK <-> 1, BAD_SIG <-> 0, MALFORMED_SIG <-> -1, BAD_KEY <-> key rejected.
Catalogue: SURVEY.md §8(d) C3 (DER malformations, r/s = 0, >= n, negative,
bit flips, off-curve keys, high-S accepted, compressed keys) plus x(P) >= n.
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, HERE)
import bc_ecdsa as ec  # noqa: E402
import openssl_ecdsa as ossl  # noqa: E402

rng = random.Random(0xC0DA0003)
vectors = []
UNPINNED = {"key_infinity", "key_hybrid"}
# OpenSSL's ECDSA_SIG uses a non-negative BIGNUM type (negative INTEGER -> decode error, -1);
# BC 1.57's ASN1Integer accepts it and ECDSASigner returns false (r < 1): BAD_SIG. Recorded, not asserted.
DIFFER = {"r_negative", "s_negative"}
OSSL = {ec.OK: 1, ec.BAD_SIG: 0, ec.MALFORMED_SIG: -1}


def add(cat, scheme, pub, sig, msg, note=""):
    st = ec.verify_status(scheme, pub, sig, msg)
    o = ossl.verify(scheme, pub, sig, msg) if len(msg) and len(sig) else None
    if cat not in UNPINNED and cat not in DIFFER and len(msg) and len(sig):
        if st == ec.BAD_KEY:
            assert o is None, (cat, note, st, o)
        else:
            assert o == OSSL[st], (cat, note, st, o)
    vectors.append({"cat": cat, "scheme": scheme, "pub": pub.hex(), "sig": sig.hex(), "msg": msg.hex(),
                    "status": st, "openssl": o, "note": note})


def txid(i):
    return hashlib.sha256(b"corda-amd-ecdsa-tx" + i.to_bytes(8, "little")).digest()


for scheme in (2, 3):
    c = ec.CURVES[scheme]
    n = c.n
    for i in range(40):
        d = rng.randrange(1, n)
        pub = ec.keypair(scheme, d)
        m = txid(scheme * 1000 + i)
        r, s = ec.sign(scheme, d, m, rng.randrange(1, n))
        sig = ec.der_encode(r, s)
        add("valid", scheme, pub, sig, m)
        add("valid_compressed", scheme, ec.compress(pub), sig, m)
        add("high_s", scheme, pub, ec.der_encode(r, n - s), m, note="n - s also verifies (no low-S rule)")
        # corruption
        b = bytearray(sig); j = rng.randrange(4, len(sig)); b[j] ^= 1 << rng.randrange(8)
        add("sig_bitflip", scheme, pub, bytes(b), m)
        mm = bytearray(m); mm[rng.randrange(32)] ^= 1 << rng.randrange(8)
        add("msg_bitflip", scheme, pub, sig, bytes(mm))
        kb = bytearray(pub); kb[1 + rng.randrange(64)] ^= 1 << rng.randrange(8)
        add("key_bitflip", scheme, bytes(kb), sig, m, note="almost surely off-curve")
        if i < 8:
            add("r_zero", scheme, pub, ec.der_encode(0, s), m)
            add("s_zero", scheme, pub, ec.der_encode(r, 0), m)
            add("r_ge_n", scheme, pub, ec.der_encode(r + n, s), m)
            add("s_ge_n", scheme, pub, ec.der_encode(r, s + n), m)
            add("r_eq_n", scheme, pub, ec.der_encode(n, s), m)
            add("r_negative", scheme, pub, ec.der_encode(-r, s), m)
            add("s_negative", scheme, pub, ec.der_encode(r, -s), m)
            add("r_n_minus_1", scheme, pub, ec.der_encode(n - 1, s), m)
            body = ec._der_int(r) + ec._der_int(s)
            add("der_long_len", scheme, pub, b"\x30\x81" + bytes([len(body)]) + body, m)
            add("der_trailing", scheme, pub, sig + b"\x00", m)
            add("der_truncated", scheme, pub, sig[:-1], m)
            add("der_indefinite", scheme, pub, b"\x30\x80" + body + b"\x00\x00", m)
            ri = ec._der_int(r)
            nonmin = b"\x02" + bytes([ri[1] + 1]) + b"\x00" + ri[2:] if ri[2] < 0x80 else b"\x02" + bytes([ri[1] + 1]) + b"\x00" + ri[2:]
            b2 = nonmin + ec._der_int(s)
            add("der_nonminimal_int", scheme, pub, b"\x30" + bytes([len(b2)]) + b2, m, note="extra leading zero")
            add("der_wrong_tag", scheme, pub, b"\x30" + bytes([len(body)]) + b"\x04" + body[1:], m)
            add("der_three_ints", scheme, pub, b"\x30" + bytes([len(body) + 3]) + body + b"\x02\x01\x01", m)
            add("der_one_int", scheme, pub, b"\x30" + bytes([len(ri)]) + ri, m)
            add("der_zero_len_int", scheme, pub, b"\x30" + bytes([2 + len(ec._der_int(s))]) + b"\x02\x00" + ec._der_int(s), m)
            add("der_bad_seq_tag", scheme, pub, b"\x31" + sig[1:], m)
            add("der_int_len_overrun", scheme, pub, sig[:3] + bytes([sig[3] + 1]) + sig[4:], m)
            add("wrong_key", scheme, ec.keypair(scheme, rng.randrange(1, n)), sig, m)
    # keys: coordinates >= p, off-curve, non-residue compressed x, infinity, hybrid, bad lengths
    d = rng.randrange(1, n)
    pub = ec.keypair(scheme, d)
    m = txid(scheme * 1000 + 999)
    r, s = ec.sign(scheme, d, m, rng.randrange(1, n))
    sig = ec.der_encode(r, s)
    x = int.from_bytes(pub[1:33], "big")
    y = int.from_bytes(pub[33:], "big")
    xs2 = 1
    while True:  # a curve point with a tiny x, so that x + p still fits 32 bytes
        rhs = (xs2 ** 3 + c.a * xs2 + c.b) % c.p
        ys2 = pow(rhs, (c.p + 1) // 4, c.p)
        if ys2 * ys2 % c.p == rhs:
            break
        xs2 += 1
    add("key_small_x", scheme, b"\x04" + xs2.to_bytes(32, "big") + ys2.to_bytes(32, "big"), sig, m)
    add("key_x_ge_p", scheme, b"\x04" + (xs2 + c.p).to_bytes(32, "big") + ys2.to_bytes(32, "big"), sig, m)
    add("key_y_plus_p", scheme, b"\x04" + pub[1:33] + ((y + c.p) % 2**256).to_bytes(32, "big"), sig, m)
    add("key_off_curve", scheme, b"\x04" + pub[1:33] + ((y + 1) % c.p).to_bytes(32, "big"), sig, m)
    xs = 1
    while True:
        rhs = (xs ** 3 + c.a * xs + c.b) % c.p
        if pow(rhs, (c.p - 1) // 2, c.p) == c.p - 1:
            break
        xs += 1
    add("key_compressed_nonresidue", scheme, b"\x02" + xs.to_bytes(32, "big"), sig, m)
    add("key_infinity", scheme, b"\x00", sig, m)
    add("key_hybrid", scheme, bytes([6 + (y & 1)]) + pub[1:], sig, m)
    add("key_len", scheme, pub[:64], sig, m)
    add("empty", scheme, pub, b"", m)
    add("empty", scheme, pub, sig, b"")
    # x(P) >= n: pick R with x in [n, p), solve for the key Q so that u1 G + u2 Q = R
    if c.p - c.n > 1000:
        xr = c.n + 1
        while True:
            rhs = (xr ** 3 + c.a * xr + c.b) % c.p
            yr = pow(rhs, (c.p + 1) // 4, c.p)
            if yr * yr % c.p == rhs:
                break
            xr += 1
        R = (xr, yr)
        rr = xr - c.n
        for t in range(3):
            m = txid(scheme * 1000 + 900 + t)
            e = int.from_bytes(hashlib.sha256(m).digest(), "big")
            ss = rng.randrange(1, n)
            w = pow(ss, n - 2, n)
            u1, u2 = e * w % n, rr * w % n
            negG = ec._mul(c, n - u1, c.G)
            Q = ec._mul(c, pow(u2, n - 2, n), ec._add(c, R, negG))
            qpub = b"\x04" + Q[0].to_bytes(32, "big") + Q[1].to_bytes(32, "big")
            add("x_ge_n", scheme, qpub, ec.der_encode(rr, ss), m, note="accept via x(P) mod n == r")
            add("x_ge_n", scheme, qpub, ec.der_encode(xr, ss), m, note="r = x(P) itself >= n: reject")

with open(os.path.join(HERE, "ecdsa_vectors.json"), "w") as f:
    json.dump({"generator": "tests/golden/make_ecdsa_vectors.py",
               "oracle": "oracle/bc_ecdsa.py (BouncyCastle 1.57 SHA256withECDSA restatement)",
               "independent": "OpenSSL 3 ECDSA_verify", "vectors": vectors}, f, indent=0)
from collections import Counter
print(len(vectors), Counter((v["cat"], v["status"]) for v in vectors if v["scheme"] == 3))
