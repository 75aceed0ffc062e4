"""The GPU Kryo encoder's template scheme, checked on the host (CPU suite).

cordahip_kryo_encode_device writes each leaf from its shape's template: the
symbols of ONE representative item traced through the encoder
(corda_amd/csrc/kryo_template.hpp). That is exact only if every input the
encoder branches on or validates is part of the shape. tools/kryo_tmpl_check.cpp
(compiled here with g++ from the same headers the GPU kernels use) groups items
by shape as the GPU does, traces each shape's first item, rebuilds EVERY item of
the shape from those symbols and compares it with the direct encoder byte for
byte. Batches: the random items of test_kryo.py, families of items that share a
shape but differ in every content byte the encoder copies (keys, X.500 name
bodies, references, quantities and nonces of one varint length), name headers
and lengths that change the shape, and the C4 cash-issue corpus.
"""
import ctypes
import os
import random
import subprocess

import numpy as np
import pytest

import kryo_leaves as K
from corda_amd import _lib
from test_kryo import C, L, O, _cash_state, _key_vectors, _random_items, x500_der

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def check(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("kt") / "kryo_tmpl_check.so")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-o", so,
                           os.path.join(ROOT, "tools", "kryo_tmpl_check.cpp")])
    lib = ctypes.CDLL(so)
    lib.kryo_template_check.restype = ctypes.c_int

    def packed(blob, arr, cap_syms=1 << 16):
        arr = arr.copy()
        arr["data"] += np.uint64(blob.ctypes.data)
        return _run(arr, cap_syms)

    def run(items, cap_syms=1 << 16):
        blob, arr, has = _lib.kryo_pack(items)
        blob = np.ascontiguousarray(blob)
        arr = arr.copy()
        arr["data"] = np.where(has, arr["data"] + np.uint64(blob.ctypes.data), 0)
        return _run(arr, cap_syms)

    def _run(arr, cap_syms):
        stats = (ctypes.c_uint64 * 6)()
        rc = lib.kryo_template_check(ctypes.c_void_p(arr.ctypes.data), ctypes.c_uint64(len(arr)),
                                     ctypes.c_uint64(cap_syms), stats)
        st = dict(zip(("shapes", "templated", "direct", "invalid", "mismatches", "too_big"), list(stats)))
        assert rc == 0 and st["mismatches"] == 0, st
        return st
    run.packed = packed
    return run


def _fixups(items):
    """test_kryo's random items as kryo_pack takes them (float / double as IEEE bits)"""
    import struct
    return [(k, (struct.unpack(">i", struct.pack(">f", v))[0] if k == "float" else
                 struct.unpack(">q", struct.pack(">d", v))[0] if k == "double" else v), c) for k, v, c in items]


def _rnd(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


def _same_len_int(rng, q):
    """another quantity / nonce whose zig-zag varlong has the same length as q's"""
    m = K.varlong_zigzag(q)
    for _ in range(200):
        x = rng.randrange(-2**63, 2**63) if q < 0 else rng.randrange(0, 2 ** min(63, max(1, q.bit_length() + 1)))
        if len(K.varlong_zigzag(x)) == len(m):
            return x
    return q


def _mutate_name(rng, name):
    """same length, same 6-byte DER header, different body bytes"""
    if len(name) <= 6:
        return name
    return name[:6] + _rnd(rng, len(name) - 6)


def _mutate_party(rng, p):
    name, key, kc = p
    return (_mutate_name(rng, name), _rnd(rng, len(key)), kc)


def test_random_items(check):
    rng = random.Random(8)
    st = check(_fixups(_random_items(rng) * 3))
    assert st["templated"] > 600


def test_cash_state_families(check):
    rng = random.Random(5)
    ref_keys = [bytes.fromhex(v["A"]) for v in _key_vectors()]
    items = []
    for f in range(40):
        d = _cash_state(rng, ref_keys, big=f % 9 == 0)
        c = rng.randrange(20, 300)
        items.append(("cash_state", d, c))
        same_owner = d["owner"] is d["issuer"]
        for _ in range(12):
            v = dict(d)
            v["issuer"] = _mutate_party(rng, d["issuer"])
            v["owner"] = v["issuer"] if same_owner else _mutate_party(rng, d["owner"])
            v["notary"] = _mutate_party(rng, d["notary"])
            v["reference"] = _rnd(rng, len(d["reference"]))
            v["legal_ref"] = _rnd(rng, 32)
            v["quantity"] = _same_len_int(rng, d["quantity"])
            items.append(("cash_state", v, c))
    st = check(items)
    # every family member rebuilt from its family's template (some mutations of
    # equal owner / issuer keys or big names may start a shape of their own)
    assert st["templated"] == len(items) and st["shapes"] <= 80, st


def test_shape_changes_are_new_shapes(check):
    """lengths, name headers, key classes, owner == issuer, encumbrance: each a shape"""
    rng = random.Random(6)
    ref_keys = [bytes.fromhex(v["A"]) for v in _key_vectors()]
    d = _cash_state(rng, ref_keys)
    d["encumbrance"] = None
    variants = [d]
    name = x500_der([(O, "Bank Q"), (L, "London"), (C, "GB")])
    for iss in ((name, ref_keys[0], 45), (name, ref_keys[0], 46), (name + b"", _rnd(rng, 91), 45),
                (x500_der([(O, "Bank QQ"), (L, "London"), (C, "GB")]), ref_keys[0], 45), (b"", ref_keys[1], 45)):
        variants.append(dict(d, issuer=iss))
        variants.append(dict(d, issuer=iss, owner=iss))
    variants += [dict(d, encumbrance=0), dict(d, encumbrance=1), dict(d, encumbrance=-7), dict(d, currency="JPY"),
                 dict(d, currency="X"), dict(d, digits=0), dict(d, reference=b"\x00\x01"),
                 dict(d, quantity=0), dict(d, quantity=2**63 - 1), dict(d, quantity=127), dict(d, quantity=128)]
    # a name whose DER header is broken: no shape (the payload does not parse);
    # the direct encoder rejects these items
    variants.append(dict(d, owner=(b"\x30\x05ab" + b"x" * 10, ref_keys[0], 45)))
    items = [("cash_state", v, 52) for v in variants for _ in range(3)]
    st = check(items)
    assert st["direct"] == 3 and st["shapes"] >= 12, st  # some variants coincide with d (its own currency, quantity length)


def test_party_and_command_families(check):
    rng = random.Random(11)
    ref_keys = [bytes.fromhex(v["A"]) for v in _key_vectors()]
    items = []
    for i in range(40):
        name = x500_der([(O, "Notary Service %d" % rng.randrange(1000)), (L, rng.choice(["Zurich", "London", "NY"])),
                         (C, rng.choice(["CH", "GB", "US"]))] + ([(O, "x" * rng.randrange(100, 300))] if i % 7 == 0 else []))
        key, kc = (rng.choice(ref_keys), 45) if i % 2 else (_rnd(rng, 91), rng.randrange(20, 200))
        xc = rng.randrange(20, 200)
        for _ in range(8):
            items.append(("party", (_mutate_name(rng, name), _rnd(rng, len(key)), kc), xc))
        keys = [(45, rng.choice(ref_keys)) if rng.random() < 0.5 else (rng.randrange(20, 200), _rnd(rng, rng.choice((32, 88, 91))))
                for _ in range(rng.randrange(1, 4 if i % 11 else 12))]
        cls = rng.choice(["net.corda.contracts.asset.Cash$Commands$Issue", "net.corda.contracts.asset.Obligation$Commands$Issue",
                          "java.security.PublicKey", "Issue", "a.b$"])
        nonce = rng.randrange(-2**63, 2**63)
        ac = rng.randrange(10, 100)
        for _ in range(8):
            items.append(("issue_command", (cls, _same_len_int(rng, nonce), [(c, _rnd(rng, len(k))) for c, k in keys]), ac))
    st = check(items)
    assert st["templated"] + st["invalid"] == len(items) and st["shapes"] <= 80, st


def test_c4_corpus(check):
    """the bench's cash-issue components (corpus.cash_issue_items): all five kinds templated"""
    from corda_amd.corpus import cash_issue_items
    rng = np.random.default_rng(4)
    ntx = 2000
    blob, items, _ = cash_issue_items(rng.integers(0, 256, (ntx, 32), dtype=np.uint8),
                                      rng.integers(0, 256, (ntx, 32), dtype=np.uint8), bytes(range(32)),
                                      rng.integers(1, 10**9, ntx), rng.integers(-2**63, 2**63 - 1, ntx))
    st = check.packed(np.ascontiguousarray(blob), items.reshape(-1))
    assert st["templated"] == 5 * ntx and st["shapes"] <= 40, st


def test_too_small_template_buffer_is_reported(check):
    rng = random.Random(3)
    ref_keys = [bytes.fromhex(v["A"]) for v in _key_vectors()]
    st = check([("cash_state", _cash_state(rng, ref_keys), 52)], cap_syms=64)
    assert st["too_big"] == 1


def test_component_leaf_bound():
    """the component-level tx path sizes each id slice's leaf buffer as 4096 + 4 x payload bytes per
    component (cordahip.cpp comp_leaf_bound): every leaf of the test corpora fits it"""
    rng = random.Random(12)
    ref_keys = [bytes.fromhex(v["A"]) for v in _key_vectors()]
    items = _fixups(_random_items(rng))
    items += [("cash_state", _cash_state(rng, ref_keys, big=i % 3 == 0), 52) for i in range(60)]
    items += [("String", "\u20ac" * n, 0) for n in (1, 63, 64, 400, 3000)]
    blob, arr, has = _lib.kryo_pack(items)
    leaves = _lib.kryo_encode(items)
    for it, leaf in zip(arr, leaves):
        nb = 2 * int(it["len"]) if int(it["kind"]) in (9, 12) else int(it["len"])
        assert len(leaf) <= 4096 + 4 * nb, (int(it["kind"]), len(leaf), nb)
