"""Native Kryo leaf encoder (cordahip_kryo_encode) on the CPU:
the library's host-side encoder against the independent Python restatement of
Kryo 4.0.0's wire format (oracle/kryo_leaves.py), and against the derived leaf
fixture of PartialMerkleTreeTest.kt:22-25 ('a'..'f'.serialize(), the leaves
of tests/golden/merkle_vectors.json "ref_*"). Everything beyond the char
fixture is PARITY UNPINNED (no Kryo / JVM in this image): the bytes follow the
published format and Corda's serializers, unconfirmed by a reference output.
The GPU half (leaves -> cordahip_tx_ids -> the fixture's tx id) is in
tests/test_gpu_tx.py::test_kryo_leaves_feed_tx_ids."""
import json
import os
import random
import struct

import pytest

import kryo_leaves as K
from corda_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_char_leaves_match_the_derived_fixture():
    fixture = {t["name"]: t for t in json.load(open(os.path.join(ROOT, "tests", "golden", "merkle_vectors.json")))["txs"]}
    leaves = _lib.kryo_encode([("char", c, 0) for c in "abcdef"])
    assert [x.hex() for x in leaves] == fixture["ref_abcdef"]["leaves"]
    assert [x.hex() for x in _lib.kryo_encode([("char", "a", 0)])] == fixture["ref_one"]["leaves"]
    assert leaves[0] == b"corda\x00\x00\x01\x07\x00a"  # header, char registration 5 + 2, 'a' big-endian


def _random_items(rng):
    items = []
    strings = ["", "x", "ab", "a" * 63, "a" * 64, "b" * 200, "café", "€100", "😀 ok",
               "\u0000\u007f", "MEGA_CORP", "O=Bank A,L=London,C=GB"]
    for _ in range(400):
        k = rng.choice(["char", "short", "int", "long", "byte", "boolean", "float", "double", "String",
                        "ed25519_key", "public_key", "kotlin_object", "raw"])
        if k == "char":
            items.append((k, rng.randrange(0, 0x10000), 0))
        elif k == "short":
            items.append((k, rng.randrange(-2**15, 2**15), 0))
        elif k == "int":
            items.append((k, rng.randrange(-2**31, 2**31), 0))
        elif k == "long":
            items.append((k, rng.randrange(-2**63, 2**63), 0))
        elif k == "byte":
            items.append((k, rng.randrange(-128, 128), 0))
        elif k == "boolean":
            items.append((k, rng.randrange(2), 0))
        elif k in ("float", "double"):
            items.append((k, rng.uniform(-1e6, 1e6), 0))
        elif k == "String":
            items.append((k, rng.choice(strings) + "".join(chr(rng.randrange(32, 0x3000)) for _ in range(rng.randrange(0, 5))), 0))
        elif k == "ed25519_key":
            items.append((k, bytes(rng.getrandbits(8) for _ in range(32)), rng.randrange(0, 300)))
        elif k == "public_key":
            items.append((k, bytes(rng.getrandbits(8) for _ in range(rng.choice((88, 91, 294)))), rng.randrange(0, 300)))
        elif k == "kotlin_object":
            items.append((k, rng.choice([K.TRANSACTION_TYPE_GENERAL, "net.corda.core.contracts.TransactionType$NotaryChange",
                                         "x", "y" * 70]), 0))
        else:
            items.append((k, bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 100))), 0))
    return items


def test_encoder_matches_python_restatement():
    rng = random.Random(8)
    items = _random_items(rng)
    got = _lib.kryo_encode([(k, (struct.unpack(">i", struct.pack(">f", v))[0] if k == "float" else
                                 struct.unpack(">q", struct.pack(">d", v))[0] if k == "double" else v), c)
                            for k, v, c in items])
    for (k, v, c), g in zip(items, got):
        want = K.leaf(k, v, c)
        assert g == want, (k, v, c, g.hex(), want.hex())


def test_known_shapes():
    gen = _lib.kryo_encode([("kotlin_object", K.TRANSACTION_TYPE_GENERAL, 0)])[0]
    name = K.TRANSACTION_TYPE_GENERAL.encode()
    assert gen == b"corda\x00\x00\x01" + b"\x01\x00" + name[:-1] + bytes([name[-1] | 0x80])
    key = bytes(range(32))
    assert _lib.kryo_encode([("ed25519_key", key, 77)])[0] == b"corda\x00\x00\x01" + bytes([79, 32]) + key
    assert _lib.kryo_encode([("ed25519_key", key, 200)])[0][8:10] == bytes([0xCA, 0x01])  # varint(202)
    assert _lib.kryo_encode([("String", "", 0), ("String", "a", 0), ("String", "ab", 0)]) == [
        b"corda\x00\x00\x01\x03\x81", b"corda\x00\x00\x01\x03\x82a", b"corda\x00\x00\x01\x03a\xe2"]
    assert _lib.kryo_encode([("int", 1, 0), ("long", -1, 0)]) == [
        b"corda\x00\x00\x01\x02\x00\x00\x00\x01", b"corda\x00\x00\x01\x09" + b"\xff" * 8]


def test_bad_items_are_rejected():
    with pytest.raises(_lib.EngineError):
        _lib.kryo_encode([("ed25519_key", b"short", 3)])
    with pytest.raises(_lib.EngineError):
        _lib.kryo_encode([("public_key", b"", 3)])


def _key_vectors():
    with open(os.path.join(ROOT, "tests", "golden", "kryo_key_vectors.json")) as f:
        return json.load(f)["vectors"]


def test_reference_ed25519_key_serialisations_pin_the_key_leaf():
    """The two Base58 party keys of samples/irs-demo/.../trade.json:3,25 are the
    reference's own p2p Kryo bytes of an EdDSAPublicKey (PublicKey.toBase58String,
    EncodingUtils.kt:67; tests/golden/make_kryo_key_vectors.py). With references
    on they read header || varint(45+2) || 01 || varint(32) || A; the Merkle
    leaf of the same key is hashed withoutReferences (Kryo.kt:550), i.e. without
    the 01 marker, which is what CORDAHIP_KRYO_ED25519_KEY with class id 45 writes."""
    vs = _key_vectors()
    assert len(vs) == 2
    alphabet = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"  # Base58.java:31
    for v in vs:
        raw = bytes.fromhex(v["serialized"])
        # the fixture's bytes are the Base58 string's: re-encode them
        x, s = int.from_bytes(raw, "big"), ""
        while x:
            x, r = divmod(x, 58)
            s = alphabet[r] + s
        assert s == v["base58"]
        A = bytes.fromhex(v["A"])
        assert raw == K.HEADER + bytes([v["class_id"] + 2, 0x01, 32]) + A
        leaf = _lib.kryo_encode([("ed25519_key", A, v["class_id"])])[0]
        assert leaf.hex() == v["leaf_without_references"]
        assert leaf == K.leaf("ed25519_key", A, v["class_id"])
        assert leaf == raw[:9] + raw[10:]  # the same bytes minus the reference marker


def test_reference_ed25519_keys_decode_in_both_oracles(oracle):
    """A5 on two reference-made keys: they decode under the i2p 0.2.0 rules (so
    arbitrary signatures are BAD_SIG, not BAD_KEY) in the C and Python oracles."""
    import i2p_ed25519 as E
    for v in _key_vectors():
        A = bytes.fromhex(v["A"])
        assert E.decode_i2p(A) is not None and E.encode(E.decode_i2p(A)) == A
        for s in v["signatures"]:
            sig, msg = bytes.fromhex(s["sig"]), bytes.fromhex(s["msg"])
            assert s["status"] == 1
            assert oracle.oracle_ed25519_verify(A, 32, sig, 64, msg, 32) == s["status"]
            assert E.verify_status(A, sig, msg) == s["status"]


def _der(tag, body):
    n = len(body)
    if n < 128:
        return bytes([tag, n]) + body
    nb = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([tag, 0x80 | len(nb)]) + nb + body


def x500_der(rdns):
    """DER of an X.500 name from (oid bytes, value) pairs, one attribute per RDN,
    values as UTF8String (BouncyCastle's default for O / L) or PrintableString (C)."""
    out = b""
    for oid, val in rdns:
        tag = 0x13 if oid == bytes([0x55, 0x04, 0x06]) else 0x0C
        out += _der(0x31, _der(0x30, _der(0x06, oid) + _der(tag, val.encode())))
    return _der(0x30, out)


O, L, C = bytes([0x55, 0x04, 0x0A]), bytes([0x55, 0x04, 0x07]), bytes([0x55, 0x04, 0x06])


def test_party_and_issue_command_leaves_match_the_restatement():
    """§8f-4 beyond keys and objects: the notary Party and the issue Command of a
    cash-issue transaction (CashIssueFlow.kt:52-54 -> OnLedgerAsset.generateIssue,
    TransactionBuilder.addCommand) natively, vs oracle/kryo_leaves.py. PARITY
    UNPINNED beyond the key bytes inside them (checked against the reference's
    own serialised key below)."""
    rng = random.Random(11)
    ref_keys = [bytes.fromhex(v["A"]) for v in _key_vectors()]
    items = []
    for i in range(120):
        name = x500_der([(O, "Notary Service %d" % rng.randrange(1000)), (L, rng.choice(["Zurich", "London", "NY"])),
                         (C, rng.choice(["CH", "GB", "US"]))] + ([(O, "x" * rng.randrange(100, 300))] if i % 7 == 0 else []))
        if i % 3 == 0:
            key, kc = rng.choice(ref_keys), 45
        elif i % 3 == 1:
            key, kc = bytes(rng.getrandbits(8) for _ in range(32)), rng.randrange(20, 200)
        else:
            key, kc = bytes(rng.getrandbits(8) for _ in range(91)), rng.randrange(20, 200)
        items.append(("party", (name, key, kc), rng.randrange(20, 200)))
        keys = [(45, rng.choice(ref_keys)) if rng.random() < 0.5 else (rng.randrange(20, 200), bytes(rng.getrandbits(8) for _ in range(rng.choice((32, 88, 91))))) for _ in range(rng.randrange(1, 4 if i % 11 else 40))]
        cls = rng.choice(["net.corda.contracts.asset.Cash$Commands$Issue", "net.corda.contracts.asset.CommodityContract$Commands$Issue",
                          "net.corda.contracts.asset.Obligation$Commands$Issue"])
        items.append(("issue_command", (cls, rng.randrange(-2**63, 2**63), keys), rng.randrange(10, 100)))
    got = _lib.kryo_encode(items)
    for (k, v, c), g in zip(items, got):
        assert g == K.leaf(k, v, c), (k, g.hex())
    # a big signer list crosses the 1024-byte chunk boundary of the signers field
    assert any(len(g) > 1100 for g in got)


def test_party_leaf_shape_with_the_reference_key():
    v = _key_vectors()[0]
    A = bytes.fromhex(v["A"])
    name = x500_der([(O, "Notary Service"), (L, "Zurich"), (C, "CH")])
    leaf = _lib.kryo_encode([("party", (name, A, v["class_id"]), 50)])[0]
    # header, NAME registration "net.corda.core.identity.Party", 2 field names,
    # then the owningKey field: one chunk holding the pinned key serialisation
    body = b"\x01\x00" + K.write_string("net.corda.core.identity.Party")
    body += b"\x02" + K.write_string("AbstractParty.owningKey") + K.write_string("Party.name")
    pinned = bytes.fromhex(v["leaf_without_references"])[8:]  # 2f 20 A
    body += bytes([len(pinned)]) + pinned + b"\x00" + bytes([1 + len(name), 52]) + name + b"\x00"
    assert leaf == K.HEADER + body


def test_issue_command_leaf_shape():
    A = bytes.fromhex(_key_vectors()[1]["A"])
    leaf = _lib.kryo_encode([("issue_command", ("net.corda.contracts.asset.Cash$Commands$Issue", -1, [(45, A)]), 10)])[0]
    assert leaf.startswith(K.HEADER + b"\x01\x00" + K.write_string("net.corda.core.contracts.Command") + b"\x02")
    assert bytes([12, 1]) + b"\x01\x01" + K.write_string("java.security.PublicKey") + b"\x2f\x20" + A in leaf
    # zig-zag(-1) = 1 in the inner chunk [01 01]; the inner endChunks flushes the
    # enclosing OutputChunked (its chunk ends there), so the inner 0 terminator is a
    # 1-byte chunk [01 00] of the value field, then the field's own 0
    assert leaf.endswith(K.write_string("Issue.nonce") + b"\x01\x01" + b"\x01\x00" + b"\x00")


def test_bad_composite_items_are_rejected():
    with pytest.raises(_lib.EngineError):
        _lib.kryo_encode([("party", (b"\x30\x40ab", b"k" * 32, 45), 50)])  # DER longer than the data
    with pytest.raises(_lib.EngineError):
        _lib.kryo_encode([("issue_command", ("net.corda.X$Issue", 1, []), 10)])  # no signers


def _party(rng, ref_keys, anonymous=False, big=False):
    name = b"" if anonymous else x500_der(
        [(O, "Bank %d" % rng.randrange(10**6)), (L, rng.choice(["London", "New York", "Zurich"])),
         (C, rng.choice(["GB", "US", "CH"]))] + ([(O, "y" * rng.randrange(900, 1500))] if big else []))
    if rng.random() < 0.5:
        return (name, rng.choice(ref_keys), 45)
    return (name, bytes(rng.getrandbits(8) for _ in range(rng.choice((32, 32, 91)))), rng.randrange(20, 300))


def _cash_state(rng, ref_keys, big=False):
    issuer = _party(rng, ref_keys, anonymous=rng.random() < 0.1, big=big and rng.random() < 0.5)
    owner = issuer if rng.random() < 0.2 else _party(rng, ref_keys, anonymous=rng.random() < 0.5,
                                                         big=big and rng.random() < 0.5)
    code, digits = rng.choice([("USD", 2), ("GBP", 2), ("JPY", 0), ("CHF", 2), ("BHD", 3), ("XAU", -1)])
    return {"quantity": rng.choice([0, 1, 100, 12345, 2**40, 2**63 - 1, rng.randrange(2**63)]),
            "currency": code, "digits": digits, "issuer": issuer,
            "reference": bytes(rng.getrandbits(8) for _ in range(rng.choice((1, 1, 2, 8, 32, 200 if big else 3)))),
            "owner": owner, "notary": _party(rng, ref_keys, big=big and rng.random() < 0.3),
            "legal_ref": K.cash_legal_ref(), "encumbrance": None if rng.random() < 0.8 else rng.randrange(-5, 2**31)}


def test_cash_state_leaf_matches_the_restatement():
    """§8f-4's last leaf: TransactionState<Cash.State> natively (CORDAHIP_KRYO_CASH_STATE)
    vs the Output/OutputChunked model of oracle/kryo_leaves.py, over Party and
    AnonymousParty owners / issuers, equal owner and issuer keys (a one-element
    exitKeys set), currencies with 0..3 and -1 fraction digits, encumbrances, and
    X.500 names long enough that nested fields cross the 1024-byte chunk buffers.
    PARITY UNPINNED beyond the key bytes inside (no Kryo here)."""
    rng = random.Random(40)
    ref_keys = [bytes.fromhex(v["A"]) for v in _key_vectors()]
    items = [("cash_state", _cash_state(rng, ref_keys, big=i % 9 == 0), rng.randrange(20, 300)) for i in range(150)]
    got = _lib.kryo_encode(items)
    for (k, v, c), g in zip(items, got):
        assert g == K.leaf(k, v, c), g.hex()
    assert any(len(g) > 2100 for g in got)


def test_cash_state_leaf_shape():
    """The structure of one cash output leaf, read back field by field: class names in
    graph order (TransactionState, Cash$State, BigDecimal, Issued, Party, OpaqueBytes,
    Currency, SecureHash$SHA256, LinkedHashSet, SingletonList = name ids 0..9), the
    pinned Ed25519 key serialisations inside, the amount and currency."""
    vs = _key_vectors()
    A0, A1 = (bytes.fromhex(v["A"]) for v in vs)
    notary = (x500_der([(O, "Notary Service"), (L, "Zurich"), (C, "CH")]), A1, 45)
    bank = (x500_der([(O, "Bank A"), (L, "London"), (C, "GB")]), A0, 45)
    d = {"quantity": 100000, "currency": "USD", "digits": 2, "issuer": bank, "reference": b"\x01",
         "owner": bank, "notary": notary, "legal_ref": K.cash_legal_ref(), "encumbrance": None}
    leaf = _lib.kryo_encode([("cash_state", d, 52)])[0]
    assert leaf == K.leaf("cash_state", d, 52)
    names = ["net.corda.core.contracts.TransactionState", "net.corda.contracts.asset.Cash$State",
             "java.math.BigDecimal", "net.corda.core.contracts.Issued", "net.corda.core.identity.Party",
             "net.corda.core.utilities.OpaqueBytes", "java.util.Currency", "net.corda.core.crypto.SecureHash$SHA256",
             "java.util.LinkedHashSet", "java.util.Collections$SingletonList"]
    pos = [leaf.find(bytes([1, i]) + K.write_string(n)) for i, n in enumerate(names)]
    assert all(p > 0 for p in pos) and pos == sorted(pos), pos
    pinned = bytes.fromhex(vs[0]["leaf_without_references"])[8:]  # 2f 20 A0
    assert leaf.count(pinned) == 4  # issuer party, exitKeys (owner = issuer: one element), owner, participants
    assert leaf.count(bytes.fromhex(vs[1]["leaf_without_references"])[8:]) == 1  # the notary
    assert K.write_string("USD") in leaf and bytes([0x02, 0x01, 0x04]) in leaf  # BigDecimal 1 x 10^-2
    assert K.varlong_zigzag(100000) in leaf
    assert leaf.count(bytes([1, 4])) >= 3  # Party re-used by name id 4 (owner, participants)
    assert K.write_string("AbstractParty.owningKey") in leaf and leaf.count(K.write_string("Party.name")) == 1


def test_bad_cash_state_is_rejected():
    rng = random.Random(2)
    ref_keys = [bytes.fromhex(v["A"]) for v in _key_vectors()]
    d = _cash_state(rng, ref_keys)
    _lib.kryo_encode([("cash_state", d, 52)])
    for bad in (dict(d, notary=(b"", d["notary"][1], 45)), dict(d, reference=b""), dict(d, currency=""),
                dict(d, owner=(b"\x30\x05ab", d["owner"][1], 45))):
        with pytest.raises(_lib.EngineError):
            _lib.kryo_encode([("cash_state", bad, 52)])
