"""CPU restatement (TEST INFRASTRUCTURE ONLY) of the reference's ECDSA verify path.

ORACLE HEADER: part of `oracle/` — a checker, never the product. Pure-Python
big ints: small cases only (golden vectors); oracle/c/ecdsa.c is the fast twin.

Path restated: `Crypto.isValid` for `ECDSA_SECP256K1_SHA256` (scheme id 2,
`core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:91-102`) and
`ECDSA_SECP256R1_SHA256` (id 3, `Crypto.kt:105-116`), `signatureName =
"SHA256withECDSA"` resolved to BouncyCastle `bcprov-jdk15on:1.57`
(`constants.properties:4`, `core/build.gradle:70-71`; jar not vendored, SURVEY
Appendix A.2). Steps, as BC 1.57 `DSABase.engineVerify` + `ECDSASigner`:

  1. derDecode (`StdDSAEncoder.decode`): the bytes must parse as a DER
     SEQUENCE of exactly two ASN.1 INTEGERs and equal their own DER
     re-encoding (CVE-2016-1000342 fix); INTEGER contents must be non-empty
     and minimal ("malformed integer", BC >= 1.56). Any failure ->
     SignatureException("error decoding signature bytes.") -> MALFORMED_SIG.
  2. e = SHA-256(message) as a big-endian integer (n is 256 bits: no truncation).
  3. r or s outside [1, n-1] (incl. negative INTEGERs) -> false (BAD_SIG).
  4. c = s^-1, u1 = e c, u2 = r c (mod n); P = u1 G + u2 Q;
     P = infinity -> false; accept iff x(P) mod n == r. No low-S rule.
  Key: SEC1 point (04||X||Y or 02/03||X) with coordinates < p on the curve,
  else the key decode throws before verify (BAD_KEY). Infinity (00) and
  hybrid (06/07) encodings: UNPINNED (rejected here as BAD_KEY).

Parity status: no known-answer vectors in the reference's tests;
pinned by the structural tests (round trip / `sig[0]++` rejects / empty
throws, CryptoUtilsTest.kt:123-231) and by OpenSSL 3 as an independent
implementation (same DER-strictness and range rules) on every vector.
"""
from __future__ import annotations

import hashlib

OK, BAD_SIG, MALFORMED_SIG, BAD_KEY, UNSUPPORTED, EMPTY = 0, 1, 2, 3, 4, 5


class Curve:
    def __init__(self, name, p, a, b, gx, gy, n):
        self.name, self.p, self.a, self.b, self.n = name, p, a, b, n
        self.G = (gx, gy)


P256 = Curve("secp256r1",
             0xffffffff00000001000000000000000000000000ffffffffffffffffffffffff,
             0xffffffff00000001000000000000000000000000fffffffffffffffffffffffc,
             0x5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b,
             0x6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296,
             0x4fe342e2fe1a7f9b8ee7eb4a7c0f9e162bce33576b315ececbb6406837bf51f5,
             0xffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551)
K1 = Curve("secp256k1",
           0xfffffffffffffffffffffffffffffffffffffffffffffffffffffffefffffc2f,
           0, 7,
           0x79be667ef9dcbbac55a06295ce870b07029bfcdb2dce28d959f2815b16f81798,
           0x483ada7726a3c4655da4fbfc0e1108a8fd17b448a68554199c47d08ffb10d4b8,
           0xfffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364141)
CURVES = {2: K1, 3: P256}


def _add(c, P1, P2):
    if P1 is None:
        return P2
    if P2 is None:
        return P1
    x1, y1 = P1
    x2, y2 = P2
    p = c.p
    if x1 == x2:
        if (y1 + y2) % p == 0:
            return None
        lam = (3 * x1 * x1 + c.a) * pow(2 * y1, p - 2, p) % p
    else:
        lam = (y2 - y1) * pow(x2 - x1, p - 2, p) % p
    x3 = (lam * lam - x1 - x2) % p
    return (x3, (lam * (x1 - x3) - y1) % p)


def _mul(c, k, P):
    R = None
    while k:
        if k & 1:
            R = _add(c, R, P)
        P = _add(c, P, P)
        k >>= 1
    return R


def decode_point(c, enc: bytes):
    """BC ECCurve.decodePoint + validation (coordinates < p, on curve)."""
    p = c.p
    if len(enc) == 65 and enc[0] == 4:
        x, y = int.from_bytes(enc[1:33], "big"), int.from_bytes(enc[33:], "big")
        if x >= p or y >= p or (y * y - x * x * x - c.a * x - c.b) % p:
            return None
        return (x, y)
    if len(enc) == 33 and enc[0] in (2, 3):
        x = int.from_bytes(enc[1:], "big")
        if x >= p:
            return None
        rhs = (x * x * x + c.a * x + c.b) % p
        y = pow(rhs, (p + 1) // 4, p)  # p = 3 mod 4 for both curves
        if y * y % p != rhs:
            return None
        if (y & 1) != (enc[0] & 1):
            y = (p - y) % p
        return (x, y)
    return None


def der_decode(sig: bytes):
    """BC 1.57 StdDSAEncoder.decode: returns (r, s) or None (malformed)."""
    def read_len(b, i):
        if i >= len(b):
            return None, i
        l0 = b[i]
        i += 1
        if l0 < 0x80:
            return l0, i
        nb = l0 & 0x7F
        if nb == 0 or nb > 4 or i + nb > len(b):
            return None, i  # indefinite / oversized
        v = int.from_bytes(b[i:i + nb], "big")
        return v, i + nb

    if len(sig) < 2 or sig[0] != 0x30:
        return None
    ln, i = read_len(sig, 1)
    if ln is None or i + ln != len(sig):  # trailing bytes / truncated
        return None
    vals = []
    end = i + ln
    while i < end:
        if sig[i] != 0x02:
            return None  # not an INTEGER (ClassCastException in BC)
        l, j = read_len(sig, i + 1)
        if l is None or j + l > end:
            return None
        body = sig[j:j + l]
        if l == 0:
            return None  # zero-length BigInteger
        if l > 1 and ((body[0] == 0 and body[1] < 0x80) or (body[0] == 0xFF and body[1] >= 0x80)):
            return None  # "malformed integer"
        vals.append(int.from_bytes(body, "big", signed=True))
        i = j + l
    if len(vals) != 2:
        return None
    r, s = vals
    # equal to its own DER re-encoding: definite minimal lengths
    if der_encode(r, s) != sig:
        return None
    return r, s


def _der_int(v: int) -> bytes:
    if v == 0:
        body = b"\x00"
    else:
        nb = (v.bit_length() + 8) // 8 if v > 0 else ((-v - 1).bit_length() + 8) // 8
        body = v.to_bytes(nb, "big", signed=True)
    return b"\x02" + _der_len(len(body)) + body


def _der_len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def der_encode(r: int, s: int) -> bytes:
    body = _der_int(r) + _der_int(s)
    return b"\x30" + _der_len(len(body)) + body


def verify_status(scheme: int, pub: bytes, sig: bytes, msg: bytes, is_valid: bool = False) -> int:
    """Crypto.doVerify semantics (Crypto.kt:472-483) by default; is_valid=True gives
    Crypto.isValid (:534-541), which has no emptiness checks (the empty message is
    hashed, an empty signature fails DER decoding)."""
    c = CURVES.get(scheme)
    if c is None:
        return UNSUPPORTED
    Q = decode_point(c, pub)  # key decode precedes doVerify's checks
    if Q is None:
        return BAD_KEY
    if not is_valid and (len(sig) == 0 or len(msg) == 0):
        return EMPTY
    rs = der_decode(sig)
    if rs is None:
        return MALFORMED_SIG
    r, s = rs
    n = c.n
    if not (1 <= r < n and 1 <= s < n):
        return BAD_SIG
    e = int.from_bytes(hashlib.sha256(msg).digest(), "big")
    w = pow(s, n - 2, n)
    P = _add(c, _mul(c, e * w % n, c.G), _mul(c, r * w % n, Q))
    if P is None:
        return BAD_SIG
    return OK if P[0] % n == r else BAD_SIG


def keypair(scheme: int, d: int):
    c = CURVES[scheme]
    Q = _mul(c, d, c.G)
    return b"\x04" + Q[0].to_bytes(32, "big") + Q[1].to_bytes(32, "big")


def compress(pub65: bytes) -> bytes:
    return bytes([2 + (pub65[64] & 1)]) + pub65[1:33]


def sign(scheme: int, d: int, msg: bytes, k: int):
    """Plain ECDSA signing with a caller-chosen nonce k (test data only)."""
    c = CURVES[scheme]
    e = int.from_bytes(hashlib.sha256(msg).digest(), "big")
    R = _mul(c, k, c.G)
    r = R[0] % c.n
    s = pow(k, c.n - 2, c.n) * (e + r * d) % c.n
    return r, s
