"""CPU restatement (TEST INFRASTRUCTURE ONLY) of the reference's Ed25519 verify path.

ORACLE HEADER
-------------
This module is part of `oracle/`: it is a checker, never the product. Only
`tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import it. Pure-Python big-int loops: use it for SMALL cases only (golden
vector generation, edge-case catalogue); `oracle/c/` is the fast restatement.

Path restated: `Crypto.doVerify/isValid` for `EDDSA_ED25519_SHA512`
(reference `core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:472-483`,
`:534-541`, scheme `:119-132`) which dispatches to the third-party engine
`net.i2p.crypto:eddsa:0.2.0` (`build.gradle:48`, `core/build.gradle:67`).
That jar is NOT in /root/reference (no Maven cache, no network), so its
published algorithm is restated here step by step:

  * key decode      = i2p `GroupElement(Curve, byte[])` (ref10 `ge_frombytes`),
                      reached via `EdDSAPublicKeySpec(A, spec)` from Corda's
                      key serializer (`core/.../serialization/Kryo.kt:389-392`)
  * hashed key      = `EdDSAPublicKey.Abyte = A.toByteArray()` (canonical)
  * verify          = i2p `EdDSAEngine.engineVerify`: |sig| == 64,
                      h = SHA-512(R || Abyte || M) mod L (no S < L check),
                      R' = B.doubleScalarMultiplyVariableTime(-A, h, S)
                      using `GroupElement.slide()` recoding, encode(R') == R
                      byte-for-byte (cofactorless).
  * slide()         = ref10 `slide`, INCLUDING the silent drop of a carry out
                      of bit 255 (the effective scalar becomes S - 2^256).

Parity status: the reference's own tests hold no known-answer vectors for
this path. The restatement is pinned by (i) the reference's
structural tests (round trip, 1-bit corruption rejects, empty input throws:
`core/src/test/kotlin/net/corda/core/crypto/CryptoUtilsTest.kt:233-286`) and
(ii) OpenSSL 3.0.2 as an independent implementation on the valid path and on
every case where RFC 8032 and i2p 0.2.0 agree. Edge semantics that only i2p
defines (S >= L, slide overflow, y >= p keys) are "parity unpinned" beyond
this restatement and its C twin agreeing.
"""
from __future__ import annotations

import hashlib
from typing import Optional, Tuple

# --- lane status codes (C-ABI contract, include/cordahip.h) -----------------
OK, BAD_SIG, MALFORMED_SIG, BAD_KEY, UNSUPPORTED, EMPTY = 0, 1, 2, 3, 4, 5

# --- curve constants (RFC 8032 §5.1; i2p `Ed25519` named curve table) -------
P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)  # i2p `curve.getI()`
_BY = (4 * pow(5, P - 2, P)) % P


def _recover_x(y: int, sign: int) -> int:
    xx = (y * y - 1) * pow(D * y * y + 1, P - 2, P) % P
    x = pow(xx, (P + 3) // 8, P)
    if (x * x - xx) % P != 0:
        x = x * SQRT_M1 % P
    if x & 1 != sign:
        x = P - x
    return x


_BX = _recover_x(_BY, 0)
# extended coordinates (X, Y, Z, T) with x = X/Z, y = Y/Z, xy = T/Z
B_POINT = (_BX, _BY, 1, _BX * _BY % P)
IDENTITY = (0, 1, 1, 0)


# --- group law (twisted Edwards a = -1; complete formulas) -------------------
def pt_add(p1, p2):
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    A = (Y1 - X1) * (Y2 - X2) % P
    Bv = (Y1 + X1) * (Y2 + X2) % P
    C = T1 * D2 % P * T2 % P
    Dv = Z1 * 2 * Z2 % P
    E, F, G, H = Bv - A, Dv - C, Dv + C, Bv + A
    return (E * F % P, G * H % P, F * G % P, E * H % P)


def pt_neg(p):
    X, Y, Z, T = p
    return ((-X) % P, Y, Z, (-T) % P)


def pt_dbl(p):
    return pt_add(p, p)


def encode(p) -> bytes:
    """i2p `GroupElement.toByteArray()` (ref10 `ge_tobytes`): canonical y, sign of x."""
    X, Y, Z, _ = p
    zi = pow(Z, P - 2, P)
    x, y = X * zi % P, Y * zi % P
    b = bytearray(y.to_bytes(32, "little"))
    b[31] |= (x & 1) << 7
    return bytes(b)


def decode_i2p(s: bytes):
    """i2p 0.2.0 `GroupElement(Curve, byte[] s)` (ref10 `ge_frombytes_negate_vartime` sans negate).

    y = s with bit 255 cleared and NOT range checked (fromByteArray reduces mod p),
    x = u v^3 (u v^7)^((p-5)/8); v x^2 == u ok, == -u -> x *= sqrt(-1), else
    IllegalArgumentException("not a valid GroupElement"); x negated when its parity
    differs from bit 255 (x == 0 with bit 255 set is accepted: -0 == 0).
    Returns None on the exception (status BAD_KEY).
    """
    if len(s) != 32:
        return None  # EdDSAPublicKeySpec: "public-key length is wrong"
    y = (int.from_bytes(s, "little") & ((1 << 255) - 1)) % P
    yy = y * y % P
    u = (yy - 1) % P
    v = (yy * D + 1) % P
    v3 = v * v % P * v % P
    x = v3 * v3 % P * v % P * u % P
    x = pow(x, (P - 5) // 8, P)
    x = v3 * u % P * x % P
    vxx = x * x % P * v % P
    if (vxx - u) % P != 0:
        if (vxx + u) % P != 0:
            return None
        x = x * SQRT_M1 % P
    if (x & 1) != ((s[31] >> 7) & 1):
        x = (-x) % P
    return (x, y, 1, x * y % P)


def slide(a: bytes) -> list:
    """i2p `GroupElement.slide(byte[])` (== ref10 `slide`), literal transcription.

    NOTE the carry loop `for k in range(i+b, 256)` silently drops a carry that
    runs past bit 255; callers get digits summing to a - 2^256 in that case.
    """
    r = [(a[i >> 3] >> (i & 7)) & 1 for i in range(256)]
    for i in range(256):
        if r[i]:
            b = 1
            while b <= 6 and i + b < 256:
                if r[i + b]:
                    if r[i] + (r[i + b] << b) <= 15:
                        r[i] += r[i + b] << b
                        r[i + b] = 0
                    elif r[i] - (r[i + b] << b) >= -15:
                        r[i] -= r[i + b] << b
                        for k in range(i + b, 256):
                            if not r[k]:
                                r[k] = 1
                                break
                            r[k] = 0
                    else:
                        break
                b += 1
    return r


def slide_value(a: bytes) -> int:
    """Integer the slide() digits represent (a, or a - 2^256 on carry drop)."""
    return sum(d << i for i, d in enumerate(slide(a)))


def _odd_multiples(p):
    """i2p `precompute(false)`: dblPrecmp = P, 3P, 5P, ..., 15P."""
    out = [p]
    p2 = pt_dbl(p)
    for _ in range(7):
        out.append(pt_add(out[-1], p2))
    return out


_B_TABLE = _odd_multiples(B_POINT)


def double_scalar_mult_vartime(a_neg, h: bytes, s: bytes):
    """i2p `B.doubleScalarMultiplyVariableTime(Aneg, h, S)` = [h](Aneg) + [S]B.

    Same loop shape as i2p: skip leading zero digits, then per position
    dbl, +/- Aneg.dblPrecmp[|d|/2], +/- B.dblPrecmp[|d|/2].
    """
    aslide, bslide = slide(h), slide(s)
    a_tab = _odd_multiples(a_neg)
    r = IDENTITY
    i = 255
    while i >= 0 and aslide[i] == 0 and bslide[i] == 0:
        i -= 1
    while i >= 0:
        t = pt_dbl(r)
        if aslide[i] > 0:
            t = pt_add(t, a_tab[aslide[i] // 2])
        elif aslide[i] < 0:
            t = pt_add(t, pt_neg(a_tab[(-aslide[i]) // 2]))
        if bslide[i] > 0:
            t = pt_add(t, _B_TABLE[bslide[i] // 2])
        elif bslide[i] < 0:
            t = pt_add(t, pt_neg(_B_TABLE[(-bslide[i]) // 2]))
        r = t
        i -= 1
    return r


def verify_status(pub: bytes, sig: bytes, msg: bytes, is_valid: bool = False) -> int:
    """Per-lane status of Crypto.isValid/doVerify for EDDSA_ED25519_SHA512.

    Order of checks follows the reference call chain:
      key decode       `Kryo.kt:389-392`    -> BAD_KEY (the key object is built when
                                               the tx is deserialised, before any verify)
      Crypto.doVerify  `Crypto.kt:474-476`  -> EMPTY for empty sig / clear data
      EdDSAEngine      sig length != 64     -> MALFORMED_SIG (SignatureException)
      math mismatch                          -> BAD_SIG (isValid false)
    """
    A = decode_i2p(pub)
    if A is None:
        return BAD_KEY
    if not is_valid and (len(sig) == 0 or len(msg) == 0):  # is_valid: Crypto.isValid has no such check
        return EMPTY
    if len(sig) != 64:
        return MALFORMED_SIG
    abyte = encode(A)
    h = int.from_bytes(hashlib.sha512(sig[:32] + abyte + msg).digest(), "little") % L
    r = double_scalar_mult_vartime(pt_neg(A), h.to_bytes(32, "little"), sig[32:])
    return OK if encode(r) == sig[:32] else BAD_SIG


def is_valid(pub: bytes, sig: bytes, msg: bytes) -> bool:
    return verify_status(pub, sig, msg) == OK


# --- RFC 8032 signing (test-data generation; mirrors Crypto.doSign for Ed25519) --
def scalar_mult(k: int, p=B_POINT):
    r = IDENTITY
    while k > 0:
        if k & 1:
            r = pt_add(r, p)
        p = pt_dbl(p)
        k >>= 1
    return r


def seed_to_keypair(seed: bytes) -> Tuple[bytes, int, bytes]:
    """i2p `EdDSAPrivateKeySpec(seed)`: h = SHA-512(seed), a = clamp(h[0:32])."""
    assert len(seed) == 32
    h = hashlib.sha512(seed).digest()
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    pub = encode(scalar_mult(a))
    return pub, a, h[32:]


def entropy_seed(entropy: int) -> bytes:
    """Corda `deriveEdDSAKeyPairFromEntropy` (`Crypto.kt:733-739`): BigInteger.toByteArray().copyOf(32)."""
    nbytes = entropy.bit_length() // 8 + 1  # two's complement, big-endian, sign bit room
    b = entropy.to_bytes(nbytes, "big", signed=True)
    return (b + bytes(32))[:32]


def sign(seed: bytes, msg: bytes) -> Tuple[bytes, bytes]:
    pub, a, prefix = seed_to_keypair(seed)
    r = int.from_bytes(hashlib.sha512(prefix + msg).digest(), "little") % L
    R = encode(scalar_mult(r))
    h = int.from_bytes(hashlib.sha512(R + pub + msg).digest(), "little") % L
    S = (r + h * a) % L
    return pub, R + S.to_bytes(32, "little")


def small_order_points():
    """The 8 torsion points (encodings are canonical), used by the edge catalogue."""
    pts = []
    for y in (1, P - 1, 0):
        for sign in (0, 1):
            try:
                x = _recover_x(y, sign)
            except Exception:
                continue
            if (D * y * y + 1) % P and ((-x * x + y * y) - 1 - D * x * x * y * y) % P == 0:
                pts.append((x, y, 1, x * y % P))
    # order-8 points: x^2 = (1 - sqrt(1 + d^-1... )) -- found via [L]Q of random Q
    seen = {encode(p) for p in pts}
    for t in range(2, 200):
        yb = (t * t + 7) % P
        Q = decode_i2p(yb.to_bytes(32, "little"))
        if Q is None:
            continue
        T = scalar_mult(L, Q)
        for k in range(8):
            e = encode(scalar_mult(k, T))
            if e not in seen:
                seen.add(e)
                pts.append(scalar_mult(k, T))
        if len(seen) == 8:
            break
    return sorted(seen)
