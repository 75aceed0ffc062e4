#!/usr/bin/env python3
"""Generate tests/golden/cert_vectors.json: ECDSA known-answer vectors made by
the REFERENCE's own BouncyCastle path, pinning oracle/bc_ecdsa.py and K2.

Source data (read from /root/reference at generation time only; the JSON is
what travels): the dev certificates Corda ships and loads itself
(node/src/main/kotlin/net/corda/node/services/config/ConfigUtilities.kt:59,84-85):
  config/dev/corda_dev_ca.cer                                        (PEM)
  node/src/main/resources/net/corda/node/internal/certificates/cordadevcakeys.jks
  node/src/main/resources/net/corda/node/internal/certificates/cordatruststore.jks
  samples/{trader,attachment}-demo/src/main/resources/certificates/{sslkeystore,truststore}.jks
Each `ecdsa-with-SHA256` certificate is a signature made by BouncyCastle
(Corda's X509Utilities) over the DER TBSCertificate with the issuer's key, so
(issuer SEC1 point, DER signature, TBS bytes) must verify: status OK under
Crypto.isValid(ECDSA_SECP256K1_SHA256 / ECDSA_SECP256R1_SHA256, ...).

JKS (Sun "JKS" v2, magic FEEDFEED) is parsed directly: trusted-certificate
entries and the certificate chains of private-key entries are plain DER; the
(encrypted) private keys are skipped, never decrypted.

Derived vectors (expected statuses fixed by construction, BC 1.57 rules):
one-bit flips inside r / s / the TBS -> BAD_SIG; the SEC1 key compressed ->
OK; a truncated DER signature -> MALFORMED_SIG; the issuer point with x
flipped (checked off-curve here with plain integers) -> BAD_KEY. The valid
vectors are also checked with OpenSSL 3 (independent) here.

Run: python3 tests/golden/make_cert_vectors.py  (needs /root/reference)
"""
import base64
import hashlib
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import openssl_ecdsa as ossl  # noqa: E402

REF = os.environ.get("CORDA_REFERENCE", "/root/reference")
SOURCES = [
    "config/dev/corda_dev_ca.cer",
    "node/src/main/resources/net/corda/node/internal/certificates/cordadevcakeys.jks",
    "node/src/main/resources/net/corda/node/internal/certificates/cordatruststore.jks",
    "samples/trader-demo/src/main/resources/certificates/sslkeystore.jks",
    "samples/trader-demo/src/main/resources/certificates/truststore.jks",
    "samples/attachment-demo/src/main/resources/certificates/sslkeystore.jks",
    "samples/attachment-demo/src/main/resources/certificates/truststore.jks",
]
OID_ECDSA_SHA256 = "1.2.840.10045.4.3.2"
OID_EC_PUBKEY = "1.2.840.10045.2.1"
CURVE_OID = {"1.3.132.0.10": 2, "1.2.840.10045.3.1.7": 3}  # secp256k1, P-256 -> Corda scheme ids
CURVE = {  # (p, a, b) for the off-curve check of derived keys
    2: (2**256 - 2**32 - 977, 0, 7),
    3: (2**256 - 2**224 + 2**192 + 2**96 - 1, -3,
        0x5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b),
}
OK, BAD_SIG, MALFORMED_SIG, BAD_KEY = 0, 1, 2, 3


# ---- minimal DER reader ------------------------------------------------------
def tlv(b, i):
    """(tag, header_len, content_start, end) of the element at b[i]."""
    tag = b[i]
    l0 = b[i + 1]
    if l0 < 0x80:
        return tag, 2, i + 2, i + 2 + l0
    nb = l0 & 0x7F
    ln = int.from_bytes(b[i + 2:i + 2 + nb], "big")
    return tag, 2 + nb, i + 2 + nb, i + 2 + nb + ln


def children(b, start, end):
    out, i = [], start
    while i < end:
        t, _, c, e = tlv(b, i)
        out.append((t, i, c, e))
        i = e
    return out


def oid_str(body):
    vals, v = [], 0
    for x in body:
        v = (v << 7) | (x & 0x7F)
        if not x & 0x80:
            vals.append(v)
            v = 0
    first = vals[0]
    return ".".join(str(x) for x in [min(first // 40, 2), first - 40 * min(first // 40, 2)] + vals[1:])


def parse_cert(der):
    _, _, c, e = tlv(der, 0)
    tbs, alg, sigv = children(der, c, e)
    tbs_bytes = der[tbs[1]:tbs[3]]
    alg_oid = oid_str(der[children(der, alg[2], alg[3])[0][2]:children(der, alg[2], alg[3])[0][3]])
    assert der[sigv[2]] == 0, "BIT STRING with unused bits"
    sig = der[sigv[2] + 1:sigv[3]]
    f = children(der, tbs[2], tbs[3])
    k = 1 if f[0][0] == 0xA0 else 0  # [0] version
    issuer = der[f[k + 2][1]:f[k + 2][3]]
    subject = der[f[k + 4][1]:f[k + 4][3]]
    spki = f[k + 5]
    a, bits = children(der, spki[2], spki[3])
    ao = children(der, a[2], a[3])
    key_alg = oid_str(der[ao[0][2]:ao[0][3]])
    curve = oid_str(der[ao[1][2]:ao[1][3]]) if len(ao) > 1 and der[ao[1][1]] == 0x06 else None
    assert der[bits[2]] == 0
    point = der[bits[2] + 1:bits[3]]
    return {"der": der, "tbs": tbs_bytes, "sig_alg": alg_oid, "sig": sig, "issuer": issuer, "subject": subject,
            "key_alg": key_alg, "curve": curve, "point": point}


# ---- JKS / PEM ---------------------------------------------------------------
def jks_certs(data):
    assert data[:4] == b"\xfe\xed\xfe\xed", "not a JKS keystore"
    _, count = struct.unpack(">II", data[4:12])
    i, out = 12, []

    def utf(i):
        n = struct.unpack(">H", data[i:i + 2])[0]
        return data[i + 2:i + 2 + n].decode(), i + 2 + n

    def cert(i):
        ctype, i = utf(i)
        assert ctype == "X.509", ctype
        n = struct.unpack(">I", data[i:i + 4])[0]
        return data[i + 4:i + 4 + n], i + 4 + n

    for _ in range(count):
        tag = struct.unpack(">I", data[i:i + 4])[0]
        alias, i = utf(i + 4)
        i += 8  # creation date
        if tag == 1:  # private key entry: skip the encrypted key, keep the chain
            n = struct.unpack(">I", data[i:i + 4])[0]
            i += 4 + n
            chain = struct.unpack(">I", data[i:i + 4])[0]
            i += 4
            for k in range(chain):
                d, i = cert(i)
                out.append((alias + "/chain%d" % k, d))
        elif tag == 2:
            d, i = cert(i)
            out.append((alias, d))
        else:
            raise ValueError("JKS entry tag %d" % tag)
    return out


def pem_certs(text):
    out, cur = [], None
    for line in text.splitlines():
        if "BEGIN CERTIFICATE" in line:
            cur = []
        elif "END CERTIFICATE" in line:
            out.append(base64.b64decode("".join(cur)))
            cur = None
        elif cur is not None:
            cur.append(line.strip())
    return out


def compress(point):
    x, y = point[1:33], int.from_bytes(point[33:], "big")
    return bytes([2 | (y & 1)]) + x


def on_curve(scheme, point):
    p, a, b = CURVE[scheme]
    x, y = int.from_bytes(point[1:33], "big"), int.from_bytes(point[33:65], "big")
    return x < p and y < p and (y * y - (x ** 3 + a * x + b)) % p == 0


def der_int_spans(sig):
    """content spans of r and s inside a DER SEQUENCE{INTEGER, INTEGER}"""
    _, _, c, e = tlv(sig, 0)
    (_, _, rc, re), (_, _, sc, se) = [(x[0], x[1], x[2], x[3]) for x in children(sig, c, e)]
    return (rc, re), (sc, se)


def main():
    certs = {}
    for rel in SOURCES:
        path = os.path.join(REF, rel)
        data = open(path, "rb").read()
        found = [(rel, d) for d in pem_certs(data.decode())] if rel.endswith(".cer") else \
            [("%s:%s" % (rel, a), d) for a, d in jks_certs(data)]
        for where, d in found:
            h = hashlib.sha256(d).hexdigest()
            certs.setdefault(h, {"where": [], **parse_cert(d)})["where"].append(where)
    by_subject = {}
    for h, c in certs.items():
        if c["key_alg"] == OID_EC_PUBKEY and c["curve"] in CURVE_OID:
            by_subject.setdefault(c["subject"], []).append(c)
    vectors = []
    pinned = 0
    for h, c in sorted(certs.items(), key=lambda kv: kv[1]["where"][0]):
        if c["sig_alg"] != OID_ECDSA_SHA256:
            continue
        issuers = by_subject.get(c["issuer"], [])
        match = None
        for iss in issuers:  # the issuer whose key verifies (several certs may share a subject name)
            scheme = CURVE_OID[iss["curve"]]
            if ossl.verify(scheme, iss["point"], c["sig"], c["tbs"]) == 1:
                match = (iss, scheme)
                break
        if match is None:
            print("no verifying issuer for", c["where"][0], file=sys.stderr)
            continue
        iss, scheme = match
        pinned += 1
        name = c["where"][0]
        pub, sig, tbs = iss["point"], c["sig"], c["tbs"]

        def add(cat, key, s, m, status, note=""):
            vectors.append({"cat": cat, "cert": name, "scheme": scheme, "pub": key.hex(), "sig": s.hex(),
                            "msg": m.hex(), "status": status, "note": note})

        add("reference_cert", pub, sig, tbs, OK, "BC-made signature shipped by the reference; OpenSSL 3: valid")
        add("reference_cert_compressed_key", compress(pub), sig, tbs, OK, "same, SEC1 compressed issuer key")
        (rc, re), (sc, se) = der_int_spans(sig)
        for lo, hi, which in ((rc, re, "r"), (sc, se, "s")):
            for pos in (hi - 1, (lo + hi) // 2):  # low byte and a middle byte of the integer
                b = bytearray(sig)
                b[pos] ^= 0x04
                add("reference_cert_flip_" + which, pub, bytes(b), tbs, BAD_SIG,
                    "one bit of %s flipped (byte %d)" % (which, pos))
        for pos in (0, len(tbs) // 2, len(tbs) - 1):
            b = bytearray(tbs)
            b[pos] ^= 0x01
            add("reference_cert_flip_tbs", pub, sig, bytes(b), BAD_SIG, "TBS byte %d flipped" % pos)
        add("reference_cert_truncated", pub, sig[:-1], tbs, MALFORMED_SIG, "DER signature missing its last byte")
        bk = bytearray(pub)
        bk[32] ^= 0x01
        assert not on_curve(scheme, bytes(bk))
        add("reference_cert_bad_key", bytes(bk), sig, tbs, BAD_KEY, "issuer x flipped: off the curve")
        if ossl.verify(scheme, pub, sig, tbs[:-1]) != 0:
            raise AssertionError("OpenSSL accepted a truncated TBS")
    out = {
        "generator": "tests/golden/make_cert_vectors.py",
        "source": "ecdsa-with-SHA256 certificates shipped in the reference (%d distinct, %d pinned vectors)"
                  % (len(certs), pinned),
        "vectors": vectors,
    }
    with open(os.path.join(HERE, "cert_vectors.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("certificates:", len(certs), "pinned signatures:", pinned, "vectors:", len(vectors))
    for h, c in certs.items():
        print("  ", c["where"][0], c["sig_alg"], c["curve"], len(c["tbs"]))


if __name__ == "__main__":
    main()
