"""K3/K4/K5 parity on the GPU: transaction ids (WireTransaction.id) and
SignedTransaction.checkSignaturesAreValid semantics, through the C-ABI."""
import ctypes
import hashlib
import json
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ED = 4


def _golden_txs():
    path = os.path.join(os.path.dirname(__file__), "golden", "merkle_vectors.json")
    return json.load(open(path))["txs"]


def test_tx_ids_golden(engine):
    txs = _golden_txs()
    ids, st = engine.tx_ids([[bytes.fromhex(x) for x in t["leaves"]] for t in txs])
    for t, i, s in zip(txs, ids, st):
        if t["id"] is None:
            assert s == 6, t["name"]  # MerkleTreeException
        else:
            assert s == 0 and i.tobytes().hex() == t["id"], t["name"]


def test_tx_ids_random_vs_oracle(engine, oracle):
    rng = random.Random(9)
    txs = []
    for _ in range(3000):
        n = rng.choice([1, 2, 3, 5, 5, 5, 8, 9, 16, 17, 40])
        txs.append([bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 200))) for _ in range(n)])
    ids, st = engine.tx_ids(txs)
    out = ctypes.create_string_buffer(32)
    for tx, i in zip(txs, ids):
        blob = np.frombuffer(b"".join(tx) or b"\0", np.uint8).copy()
        off = np.zeros(len(tx) + 1, np.uint64)
        off[1:] = np.cumsum([len(x) for x in tx])
        assert oracle.oracle_tx_id(blob.ctypes.data, off.ctypes.data, len(tx), out) == 0
        assert out.raw == i.tobytes()
    assert (st == 0).all()


def _sign(oracle, seed, msg):
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    oracle.oracle_ed25519_sign(seed, msg, len(msg), pub, sig)
    return pub.raw, sig.raw


def test_signed_tx_semantics(engine, oracle):
    """TransactionSerializationTests.kt:61-97 / TransactionTests.kt:27-94 shapes."""
    rng = random.Random(4)
    txs = [[bytes(rng.getrandbits(8) for _ in range(n)) for n in (450, 150, 140, 43, 55)] for _ in range(6)]
    ids, _ = engine.tx_ids(txs)
    seeds = [hashlib.sha256(b"signer%d" % i).digest() for i in range(3)]
    good = [[(ED,) + _sign(oracle, sd, ids[t].tobytes()) for sd in seeds] for t in range(len(txs))]
    sigs = [list(g) for g in good]
    # tx1: second signature corrupted -> first_bad = 1, BAD_SIG
    s1 = bytearray(sigs[1][1][2]); s1[0] ^= 1
    sigs[1][1] = (ED, sigs[1][1][1], bytes(s1))
    # tx2: signatures swapped between transactions -> BAD_SIG at index 0
    sigs[2][0] = good[3][0]
    # tx3: one component byte changed -> the recomputed id no longer matches every signature
    txs[3][2] = bytes([txs[3][2][0] ^ 1]) + txs[3][2][1:]
    # tx4: no signatures; tx5: no components; tx6: neither (the constructor's
    # require(sigs.isNotEmpty()), SignedTransaction.kt:37-39, fires before tx.id)
    sigs[4] = []
    txs[5] = []
    txs.append([])
    sigs.append([])
    got_ids, tx_st, first_bad, sig_st = engine.signed_tx_verify(txs, sigs)
    assert list(tx_st) == [0, 1, 1, 1, 7, 6, 7]
    assert list(first_bad) == [-1, 1, 0, 0, -1, -1, -1]
    assert got_ids[0].tobytes() == ids[0].tobytes()
    flat = [x for per in sigs for x in per]
    assert len(sig_st) == len(flat)


@pytest.mark.parametrize("slices", ["default", "1", "3", "16"])
def test_signed_tx_id_slices(engine, oracle, slices, monkeypatch):
    """cordahip_signed_tx_verify with the tx ids in asynchronous slices that feed
    the signature pipeline (CORDAHIP_TX_SLICES uniform slices; the default is one
    slice per signature chunk), the signatures in 7-lane pipeline chunks
    (CORDAHIP_TX_SIG_CHUNK) that end mid-slice and mid-transaction, each gathering
    its message rows on the GPU from the ids in HBM after the slice holding its
    last transaction, each finished chunk reducing the transactions it holds
    whole: results must not depend on the slicing, including slices with no
    transactions and transactions without signatures or components."""
    if slices == "default":
        monkeypatch.delenv("CORDAHIP_TX_SLICES", raising=False)
    else:
        monkeypatch.setenv("CORDAHIP_TX_SLICES", slices)
    monkeypatch.setenv("CORDAHIP_TX_SIG_CHUNK", "7")
    rng = random.Random(31)
    txs = [[bytes(rng.getrandbits(8) for _ in range(n)) for n in (120, 60, 43)] for _ in range(150)]
    ids, _ = engine.tx_ids(txs)
    sigs = []
    for t in range(150):
        per = []
        for j in range(t % 4):
            p, s = _sign(oracle, hashlib.sha256(b"sl%d" % j).digest(), ids[t].tobytes())
            if t % 11 == 5 and j == 1:
                s = s[:3] + bytes([s[3] ^ 2]) + s[4:]
            per.append((ED, p, s))
        sigs.append(per)
    txs[7] = []  # no components
    got_ids, tx_st, first_bad, sig_st = engine.signed_tx_verify(txs, sigs)
    want = []
    for t in range(150):
        if not sigs[t]:
            want.append(7)
        elif not txs[t]:
            want.append(6)
        elif t % 11 == 5 and len(sigs[t]) > 1:
            want.append(1)
        else:
            want.append(0)
    assert [int(x) for x in tx_st] == want
    assert [int(x) for x in first_bad] == [1 if w == 1 else -1 for w in want]
    assert all(got_ids[t].tobytes() == ids[t].tobytes() for t in range(150) if t != 7)


def test_signed_tx_device_path(engine, oracle):
    torch = pytest.importorskip("torch")
    rng = random.Random(12)
    ntx = 700
    txs = [[bytes(rng.getrandbits(8) for _ in range(n)) for n in (450, 150, 140, 43, 55)] for _ in range(ntx)]
    ids, _ = engine.tx_ids(txs)
    nsig = [rng.choice([1, 2, 3]) for _ in range(ntx)]
    keys, sgs = [], []
    for t in range(ntx):
        for k in range(nsig[t]):
            p, s = _sign(oracle, hashlib.sha256(b"k%d" % ((t * 7 + k) % 50)).digest(), ids[t].tobytes())
            if t % 10 == 3 and k == nsig[t] - 1:
                s = s[:40] + bytes([s[40] ^ 4]) + s[41:]
            keys.append(p)
            sgs.append(s)
    dev = torch.device("cuda:0")
    leaves = [x for tx in txs for x in tx]
    lb = torch.tensor(np.frombuffer(b"".join(leaves), np.uint8), device=dev)
    lo = torch.tensor(np.concatenate([[0], np.cumsum([len(x) for x in leaves])]).astype(np.int64), device=dev)
    tlo = torch.tensor(np.arange(0, 5 * ntx + 1, 5, dtype=np.int64), device=dev)
    tso = torch.tensor(np.concatenate([[0], np.cumsum(nsig)]).astype(np.int64), device=dev)
    k = torch.tensor(np.frombuffer(b"".join(keys), np.uint8).reshape(-1, 32), device=dev)
    s = torch.tensor(np.frombuffer(b"".join(sgs), np.uint8).reshape(-1, 64), device=dev)
    txid = torch.empty((ntx, 32), dtype=torch.uint8, device=dev)
    tst = torch.empty(ntx, dtype=torch.uint8, device=dev)
    fb = torch.empty(ntx, dtype=torch.int64, device=dev)
    sst = torch.empty(len(keys), dtype=torch.uint8, device=dev)
    engine.signed_tx_verify_ed25519_device(lb, lo, tlo, tso, k, s, txid, tst, fb, sst)
    torch.cuda.synchronize()
    assert np.array_equal(txid.cpu().numpy(), ids)
    want_bad = [(nsig[t] - 1 if t % 10 == 3 else -1) for t in range(ntx)]
    assert list(fb.cpu().numpy()) == want_bad
    assert list(tst.cpu().numpy()) == [1 if t % 10 == 3 else 0 for t in range(ntx)]


@pytest.mark.gpu
def test_leaf_sha256_every_length_and_alignment(engine):
    """K3's aligned-dword loader: single-leaf transactions (root = the leaf hash,
    MerkleTree.kt:51-52) of every length 0..300 packed back to back, so every
    length meets every byte alignment; checked against hashlib."""
    import hashlib
    rng = random.Random(21)
    txs = []
    for shift in range(4):
        txs.append([bytes(rng.getrandbits(8) for _ in range(shift + 1))])  # vary the running offset
        txs += [[bytes(rng.getrandbits(8) for _ in range(n))] for n in range(301)]
    ids, st = engine.tx_ids(txs)
    assert (st == 0).all()
    for t, tx in enumerate(txs):
        assert bytes(ids[t]) == hashlib.sha256(tx[0]).digest(), (t, len(tx[0]))


def test_kryo_leaves_feed_tx_ids(engine, oracle):
    """§8f rank 4: leaves made by the native Kryo encoder (cordahip_kryo_encode)
    go straight into cordahip_tx_ids. The char leaves of PartialMerkleTreeTest.kt:22-25
    give the derived fixture's ids; mixed transactions (native mustSign-key and
    TransactionType leaves beside RAW JVM-serialised ones) match the oracle's id
    over the same bytes (the native leaf bytes themselves: PARITY UNPINNED beyond
    the char fixture, tests/test_kryo.py)."""
    from corda_amd import _lib
    import kryo_leaves as K
    fixture = {t["name"]: t for t in _golden_txs()}
    txs = [_lib.kryo_encode([("char", c, 0) for c in "abcdef"]), _lib.kryo_encode([("char", "a", 0)]),
           _lib.kryo_encode([("char", c, 0) for c in "abc"])]
    rng = random.Random(3)
    for t in range(20):
        items = [("raw", b"corda\x00\x00\x01" + bytes(rng.getrandbits(8) for _ in range(n)), 0) for n in (440, 140)]
        items += [("ed25519_key", bytes(rng.getrandbits(8) for _ in range(32)), 71) for _ in range(t % 3 + 1)]
        items.append(("kotlin_object", K.TRANSACTION_TYPE_GENERAL, 0))
        txs.append(_lib.kryo_encode(items))
    ids, st = engine.tx_ids(txs)
    assert (st == 0).all()
    assert [i.tobytes().hex() for i in ids[:3]] == [fixture[n]["id"] for n in ("ref_abcdef", "ref_one", "ref_three")]
    out = ctypes.create_string_buffer(32)
    for tx, i in zip(txs[3:], ids[3:]):
        blob = np.frombuffer(b"".join(tx), np.uint8).copy()
        off = np.zeros(len(tx) + 1, np.uint64)
        off[1:] = np.cumsum([len(x) for x in tx])
        assert oracle.oracle_tx_id(blob.ctypes.data, off.ctypes.data, len(tx), out) == 0
        assert out.raw == i.tobytes()


def test_native_cash_issue_leaves_feed_tx_ids(engine, oracle):
    """§8f-4 for the C4 cash-issue shape (CashIssueFlow.kt:52-54), ALL FIVE leaves
    made natively: the TransactionState<Cash.State> output (CASH_STATE), the
    command (ISSUE_COMMAND), notary Party (PARTY), mustSign key (ED25519_KEY,
    pinned by the reference's own key serialisations) and TransactionType
    (KOTLIN_OBJECT) -- no JVM re-serialisation. Leaves in availableComponents order
    (MerkleTransaction.kt:51-62); every leaf equals oracle/kryo_leaves.py's, and the
    tx ids from cordahip_tx_ids equal the C oracle's over the same bytes."""
    from corda_amd import _lib
    import kryo_leaves as K
    from test_kryo import C, L, O, x500_der, _key_vectors
    rng = random.Random(21)
    ref = [bytes.fromhex(v["A"]) for v in _key_vectors()]
    txs = []
    notary_name = x500_der([(O, "Notary Service"), (L, "Zurich"), (C, "CH")])
    for t in range(64):
        issuer = ref[t % 2] if t % 4 < 2 else bytes(rng.getrandbits(8) for _ in range(32))
        bank = (x500_der([(O, "Bank %d" % (t % 5)), (L, "London"), (C, "GB")]), issuer, 45)
        owner = (b"", bytes(rng.getrandbits(8) for _ in range(32)), 45) if t % 3 else bank  # anonymised recipient
        notary = (notary_name, ref[(t + 1) % 2], 45)
        state = {"quantity": rng.randrange(1, 10**9), "currency": rng.choice(["USD", "GBP", "JPY"]), "digits": 2,
                 "issuer": bank, "reference": bytes([t % 256]), "owner": owner, "notary": notary,
                 "legal_ref": K.cash_legal_ref(), "encumbrance": None}
        state["digits"] = 0 if state["currency"] == "JPY" else 2
        items = [("cash_state", state, 52),
                 ("issue_command", ("net.corda.contracts.asset.Cash$Commands$Issue", rng.randrange(-2**63, 2**63),
                                    [(45, issuer)]), 10),
                 ("party", (notary_name, notary[1], 45), 52),
                 ("ed25519_key", issuer, 45),
                 ("kotlin_object", K.TRANSACTION_TYPE_GENERAL, 0)]
        leaves = _lib.kryo_encode(items)
        assert leaves == [K.leaf(k, v, c) for k, v, c in items]
        txs.append(leaves)
    ids, st = engine.tx_ids(txs)
    assert (st == 0).all()
    out = ctypes.create_string_buffer(32)
    for tx, i in zip(txs, ids):
        blob = np.frombuffer(b"".join(tx), np.uint8).copy()
        off = np.zeros(len(tx) + 1, np.uint64)
        off[1:] = np.cumsum([len(x) for x in tx])
        assert oracle.oracle_tx_id(blob.ctypes.data, off.ctypes.data, len(tx), out) == 0
        assert out.raw == i.tobytes()


def test_signed_tx_golden_edge_signatures(engine, oracle):
    """The Ed25519 golden catalogue's keys and signatures (bad keys, non-canonical
    and off-curve R, S >= L, small-order points, malformed lengths, ...) as the
    signatures of transactions, so they run through the signed-tx pipeline -- whose
    leaf batches decode keys before their ids arrive (the prep's key half, then the
    gather and the message half) -- each checked against the C oracle over its
    transaction's id; then the per-transaction first failing signature."""
    vs = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ed25519_vectors.json")))["vectors"]
    rng = random.Random(61)
    ntx = 400
    txs = [[bytes(rng.getrandbits(8) for _ in range(n)) for n in (450, 150, 140, 43, 55)] for _ in range(ntx)]
    ids, _ = engine.tx_ids(txs)
    sigs, want = [], []
    k = 0
    for t in range(ntx):
        per, st = [], []
        for _ in range(rng.choice([1, 2, 3])):
            v = vs[k % len(vs)]
            k += 1
            pub, sig = bytes.fromhex(v["pub"]), bytes.fromhex(v["sig"])
            per.append((ED, pub, sig))
            msg = ids[t].tobytes()
            st.append(oracle.oracle_ed25519_verify(pub, len(pub), sig, len(sig), msg, len(msg)))
        sigs.append(per)
        want.append(st)
    got_ids, tx_st, first_bad, sig_st = engine.signed_tx_verify(txs, sigs)
    flat_want = [x for st in want for x in st]
    assert [int(x) for x in sig_st] == flat_want
    for t in range(ntx):
        bad = [q for q, x in enumerate(want[t]) if x != 0]
        assert int(first_bad[t]) == (bad[0] if bad else -1), t
        assert int(tx_st[t]) == (want[t][bad[0]] if bad else 0), t
    assert any(x == 3 for x in flat_want) and any(x == 1 for x in flat_want)  # bad keys and bad signatures ran
