"""The product's strict DER decoder (corda_amd/csrc/der.hpp, shared by the
ECDSA prep kernel and the host runtime's long-signature path) against the
oracle's BC 1.57 StdDSAEncoder restatement (oracle/bc_ecdsa.py der_decode) on
the golden signatures, the reference's certificate signatures and ~20k
mutated / synthetic encodings. The header is compiled for the host with g++
(it is plain C++ outside HIP) into a throwaway harness."""
import ctypes
import json
import os
import random
import subprocess

import pytest

from conftest import ROOT

import sys
sys.path.insert(0, ROOT)
from oracle.bc_ecdsa import der_decode, der_encode  # noqa: E402

HARNESS = r'''
#include <stdint.h>
#include <string.h>
#include "der.hpp"
extern "C" int der_probe(const uint8_t* sig, uint32_t n, uint32_t* out /* [2][10] */) {
  cordahip::DerInt r, s;
  if (!cordahip::der_decode_sig(sig, n, r, s)) return 0;
  const cordahip::DerInt* d[2] = {&r, &s};
  for (int k = 0; k < 2; k++) {
    for (int q = 0; q < 8; q++) out[10 * k + q] = d[k]->v[q];
    out[10 * k + 8] = d[k]->neg;
    out[10 * k + 9] = d[k]->big;
  }
  return 1;
}
'''


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    d = tmp_path_factory.mktemp("der")
    src, lib = d / "der_probe.cpp", d / "der_probe.so"
    src.write_text(HARNESS)
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I", os.path.join(ROOT, "corda_amd", "csrc"),
                    "-o", str(lib), str(src)], check=True)
    so = ctypes.CDLL(str(lib))
    so.der_probe.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    so.der_probe.restype = ctypes.c_int

    def run(sig: bytes):
        out = (ctypes.c_uint32 * 20)()
        ok = so.der_probe(sig, len(sig), out)
        if not ok:
            return None
        res = []
        for k in range(2):
            v = sum(out[10 * k + q] << (32 * q) for q in range(8))
            res.append((v, bool(out[10 * k + 8]), bool(out[10 * k + 9])))
        return res
    return run


def _agree(probe, sig: bytes):
    want = der_decode(sig)
    got = probe(sig)
    assert (want is None) == (got is None), sig.hex()
    if want is None:
        return
    for x, (v, neg, big) in zip(want, got):
        assert neg == (x < 0), sig.hex()
        if x >= 0:
            assert big == (x >= 1 << 256), sig.hex()
            if not big:
                assert v == x, sig.hex()


def _corpus():
    sigs = []
    g = os.path.join(ROOT, "tests", "golden")
    for name in ("ecdsa_vectors.json", "cert_vectors.json"):
        path = os.path.join(g, name)
        if not os.path.exists(path):
            continue
        data = json.load(open(path))
        items = data if isinstance(data, list) else data.get("vectors", [])
        for v in items:
            if isinstance(v, dict) and "sig" in v:
                sigs.append(bytes.fromhex(v["sig"]))
    return sigs


def test_golden_and_certificate_signatures(probe):
    sigs = _corpus()
    assert len(sigs) > 50
    for s in sigs:
        _agree(probe, s)


def _long_len(n):
    b = n.to_bytes((n.bit_length() + 7) // 8 or 1, "big")
    return bytes([0x80 | len(b)]) + b


def test_mutations_and_synthetic_encodings(probe):
    rng = random.Random(0xDE4)
    base = _corpus()
    cases = 0
    for _ in range(12000):
        s = bytearray(rng.choice(base))
        op = rng.randrange(5)
        if op == 0 and s:
            s[rng.randrange(len(s))] ^= 1 << rng.randrange(8)
        elif op == 1 and s:
            del s[rng.randrange(len(s)):]
        elif op == 2:
            s.insert(rng.randrange(len(s) + 1), rng.randrange(256))
        elif op == 3 and len(s) > 2:
            s[1] = rng.randrange(256)
        else:
            s += bytes([rng.randrange(256)])
        _agree(probe, bytes(s))
        cases += 1
    # synthetic INTEGER bodies: leading zeros, 33-byte, 64-byte, negative, long-form lengths
    for _ in range(8000):
        def integer():
            kind = rng.randrange(6)
            if kind == 0:
                x = rng.getrandbits(rng.randrange(1, 257))
                return x, None
            if kind == 1:
                body = bytes([0]) * rng.randrange(1, 4) + rng.getrandbits(256).to_bytes(32, "big")
                return None, body
            if kind == 2:
                return None, rng.getrandbits(8 * 40).to_bytes(40, "big")  # > 32 significant bytes
            if kind == 3:
                return -rng.getrandbits(200) - 1, None
            if kind == 4:
                return None, bytes([0xff, rng.randrange(256)]) + bytes(rng.randrange(1, 5))
            return 1 << 256, None
        parts = []
        for _k in range(2):
            x, body = integer()
            if body is None:
                body = x.to_bytes((x.bit_length() + 8) // 8 or 1, "big", signed=True)
            ln = bytes([len(body)]) if len(body) < 0x80 and rng.random() < 0.9 else _long_len(len(body))
            parts.append(b"\x02" + ln + body)
        content = b"".join(parts)
        ln = bytes([len(content)]) if len(content) < 0x80 and rng.random() < 0.9 else _long_len(len(content))
        _agree(probe, b"\x30" + ln + content)
        cases += 1
    # well-formed round trips over the full range
    for _ in range(2000):
        r, s = rng.getrandbits(256), rng.getrandbits(256)
        _agree(probe, der_encode(r, s))
    assert cases == 20000
