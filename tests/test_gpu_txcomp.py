"""Component-level SignedTransaction batches (cordahip_signed_txcomp_verify /
cordahip_txcomp_submit): the JVM hands over each transaction's components as
Kryo items and the GPU writes their leaves (the template encoder) before K3/K4.

Checked against (a) the C oracle's tx ids over the Python restatement's leaves
(oracle/kryo_leaves.py), and (b) the leaf-level path (cordahip_signed_tx_verify
over the host encoder's leaves) output by output: ids, tx statuses,
first_bad_sig and every signature status -- including signatures corrupted,
transactions with a component the encoder rejects (CORDAHIP_TX_BAD_COMPONENT),
with no components (NO_LEAVES) and without signatures (NO_SIGNATURES), payloads
shared by many items, multi-slice shards and the ticketed form."""
import ctypes
import hashlib
import os
import random

import numpy as np
import pytest

import kryo_leaves as K
import test_kryo as TK
from corda_amd import _lib
from corda_amd.corpus import cash_issue_items

pytestmark = pytest.mark.gpu
ED = 4


def _sign(oracle, seed, msg):
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    oracle.oracle_ed25519_sign(seed, msg, len(msg), pub, sig)
    return pub.raw, sig.raw


def _oracle_id(oracle, leaves):
    out = ctypes.create_string_buffer(32)
    blob = np.frombuffer(b"".join(leaves) or b"\0", np.uint8).copy()
    off = np.zeros(len(leaves) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in leaves])
    rc = oracle.oracle_tx_id(blob.ctypes.data, off.ctypes.data, len(leaves), out)
    return out.raw if rc == 0 else None


def _random_txs(rng, ntx):
    """(components per tx in the restatement's form, the same in the library's form)"""
    ref_keys = [bytes.fromhex(v["A"]) for v in TK._key_vectors()]
    pool = TK._random_items(rng)
    spec = []
    for t in range(ntx):
        comps = []
        for _ in range(rng.choice([1, 2, 5, 5, 5, 7])):
            r = rng.random()
            if r < 0.3:
                comps.append(("cash_state", TK._cash_state(rng, ref_keys, big=t % 37 == 0), 52))
            elif r < 0.45:
                comps.append(("party", TK._party(rng, ref_keys), 52))
            elif r < 0.6:
                comps.append(("issue_command", ("net.corda.contracts.asset.Cash$Commands$Issue",
                                                rng.randrange(-2**63, 2**63),
                                                [(45, rng.choice(ref_keys)) for _ in range(rng.randrange(1, 4))]), 10))
            else:
                comps.append(rng.choice(pool))
        spec.append(comps)
    lib_form = [[(k, _bits(k, v), c) for k, v, c in comps] for comps in spec]
    return spec, lib_form


def _bits(k, v):
    import struct
    if k == "float":
        return struct.unpack(">i", struct.pack(">f", v))[0]
    if k == "double":
        return struct.unpack(">q", struct.pack(">d", v))[0]
    return v


def _signers(oracle, rng, ids, ntx, corrupt=0.05):
    sigs = []
    for t in range(ntx):
        per = []
        for q in range(rng.choice([0, 1, 2, 3]) if t % 50 == 7 else rng.choice([1, 2, 3])):
            pub, sg = _sign(oracle, hashlib.sha256(b"txc%d-%d" % (t, q)).digest(), ids[t] if ids[t] else b"\0" * 32)
            sg = bytearray(sg)
            if rng.random() < corrupt:
                sg[rng.randrange(64)] ^= 1 << rng.randrange(8)
            per.append((ED, pub, bytes(sg)))
        sigs.append(per)
    return sigs


def _compare(engine, leaves_per_tx, comp_result, sigs):
    """the component path's outputs == the leaf path's over the host encoder's leaves"""
    ids_l, st_l, fb_l, sst_l = engine.signed_tx_verify(leaves_per_tx, sigs)
    ids_c, st_c, fb_c, sst_c = comp_result
    assert np.array_equal(st_c, st_l)
    assert np.array_equal(fb_c, fb_l)
    assert np.array_equal(sst_c, sst_l)
    assert np.array_equal(ids_c[st_l == 0], ids_l[st_l == 0])


def test_components_vs_oracle_and_leaf_path(engine, oracle):
    rng = random.Random(51)
    ntx = 400
    spec, comps = _random_txs(rng, ntx)
    comps[3] = []  # no components: MerkleTreeException (NO_LEAVES)
    spec[3] = []
    leaves = [[K.leaf(k, v, c) for k, v, c in tx] for tx in spec]
    ids = [_oracle_id(oracle, lv) if lv else None for lv in leaves]
    sigs = _signers(oracle, rng, ids, ntx)
    res = engine.signed_txcomp_verify(comps, sigs)
    got_ids, st, fb, sst = res
    for t in range(ntx):
        if ids[t] is not None and sigs[t]:
            assert got_ids[t].tobytes() == ids[t], t
    assert st[3] == _lib.TX_NO_SIGNATURES or st[3] == _lib.TX_NO_LEAVES
    assert (st == _lib.TX_NO_SIGNATURES).sum() >= 1 and (st == 1).sum() >= 5 and (st == 0).sum() > 200
    _compare(engine, leaves, res, sigs)


def test_bad_components(engine, oracle):
    """an invalid component (cordahip_kryo_encode rejects it) or one whose payload runs past the
    payload's end: CORDAHIP_TX_BAD_COMPONENT, its signatures carry that status, first_bad -1"""
    rng = random.Random(52)
    ref_keys = [bytes.fromhex(v["A"]) for v in TK._key_vectors()]
    good = [("cash_state", TK._cash_state(rng, ref_keys), 52), ("ed25519_key", ref_keys[0], 45),
            ("kotlin_object", K.TRANSACTION_TYPE_GENERAL, 0)]
    bad = [("ed25519_key", b"k" * 31, 45)]
    txs = [good, good[:2] + bad, good, [bad[0]], good]
    leaves_ok = [K.leaf(k, v, c) for k, v, c in good]
    tid = _oracle_id(oracle, leaves_ok)
    sigs = [[(ED,) + _sign(oracle, b"\x11" * 32, tid)] for _ in txs]
    ids, st, fb, sst = engine.signed_txcomp_verify(txs, sigs)
    assert list(st) == [0, _lib.TX_BAD_COMPONENT, 0, _lib.TX_BAD_COMPONENT, 0]
    assert list(fb) == [-1] * 5 and list(sst) == [0, 9, 0, 9, 0]
    assert ids[0].tobytes() == tid and ids[4].tobytes() == tid
    # a payload offset past the end of the payload; the outputs in pageable, then in pinned
    # memory (merkle_root stores the ids and statuses through the device mapping)
    blob, items, has = _lib.kryo_pack([c for tx in txs[:1] for c in tx])
    items = items.copy()
    items["data"] = np.where(has, items["data"], 0)
    items2 = np.concatenate([items, items, items])
    items2[4]["data"] = len(blob) - 3  # the second tx's key: 32 bytes from 3 before the end
    tio = np.array([0, 3, 6, 6, 9], np.uint64)  # the third tx has no components
    for pinned in (False, True):
        ids, st, fb, sst = engine.signed_txcomp_verify_arrays(blob, items2, tio, sigs[:4], pinned_out=pinned)
        assert list(st) == [0, _lib.TX_BAD_COMPONENT, _lib.TX_NO_LEAVES, 0], pinned
        assert ids[0].tobytes() == tid and ids[3].tobytes() == tid and not ids[2].any()


@pytest.mark.parametrize("chunk", [None, "4096"])
def test_cash_issue_corpus_many_slices(engine, oracle, chunk):
    """the bench's cash-issue components (payloads shared by every transaction: the notary Party
    and TransactionType) through the component path, in one or many id slices, against the leaf
    path over the host encoder's leaves and the oracle's ids; plus the ticketed form"""
    torch = pytest.importorskip("torch")  # noqa: F841
    rng = np.random.default_rng(53)
    ntx = 12000
    ik = rng.integers(0, 256, (ntx, 32), dtype=np.uint8)
    blob, items, _ = cash_issue_items(ik, rng.integers(0, 256, (ntx, 32), dtype=np.uint8), bytes(range(32)),
                                      rng.integers(1, 10**9, ntx), rng.integers(-2**63, 2**63 - 1, ntx))
    it = items.reshape(-1).copy()
    host_it = it.copy()
    host_it["data"] += np.uint64(blob.ctypes.data)
    hb, ho = _lib.kryo_encode_array(host_it)
    leaves = [[hb[int(ho[5 * t + j]):int(ho[5 * t + j + 1])].tobytes() for j in range(5)] for t in range(ntx)]
    ids = [_oracle_id(oracle, leaves[t]) for t in range(0, ntx, 997)]
    # signatures: one per tx over the (leaf-path) id, every 10th corrupted
    ids_l, _ = engine.tx_ids(leaves)
    sigs = []
    for t in range(ntx):
        pub, sg = _sign(oracle, hashlib.sha256(b"c4c%d" % t).digest(), ids_l[t].tobytes())
        if t % 10 == 3:
            sg = sg[:5] + bytes([sg[5] ^ 4]) + sg[6:]
        sigs.append([(ED, pub, sg)] * (1 + t % 3))
    tio = np.arange(0, 5 * ntx + 1, 5, dtype=np.uint64)
    old = os.environ.get("CORDAHIP_TX_SIG_CHUNK")
    if chunk:
        os.environ["CORDAHIP_TX_SIG_CHUNK"] = chunk
    try:
        res = engine.signed_txcomp_verify_arrays(blob, it, tio, sigs)
        tk = engine.signed_txcomp_verify_arrays(blob, it, tio, sigs, async_=True, pinned_out=True)
        res2 = tk.wait()
    finally:
        if chunk:
            if old is None:
                del os.environ["CORDAHIP_TX_SIG_CHUNK"]
            else:
                os.environ["CORDAHIP_TX_SIG_CHUNK"] = old
    for a, b in zip(res, res2):
        assert np.array_equal(a, b)
    assert [res[0][t].tobytes() for t in range(0, ntx, 997)] == ids
    assert (res[1] == 0).sum() == ntx - len(range(3, ntx, 10))
    _compare(engine, leaves, res, sigs)


def test_templates_only_chain_and_its_redo(engine, oracle):
    """Once a device's component batches stop needing new templates and the direct
    encoder, the next batch runs the templates-only chain (no build / size / direct-write
    kernels); a batch that then brings new shapes (strings of lengths not seen before)
    and direct items (a 70,000-character string, beyond a template) misses and is run
    again with the full chain. Every call's outputs equal the leaf path's."""
    rng = np.random.default_rng(54)
    ntx = 3000
    blob, items, _ = cash_issue_items(rng.integers(0, 256, (ntx, 32), dtype=np.uint8),
                                      rng.integers(0, 256, (ntx, 32), dtype=np.uint8), bytes(range(32)),
                                      rng.integers(1, 10**9, ntx), rng.integers(-2**63, 2**63 - 1, ntx))
    it = items.reshape(-1).copy()
    host_it = it.copy()
    host_it["data"] += np.uint64(blob.ctypes.data)
    hb, ho = _lib.kryo_encode_array(host_it)
    cash_leaves = [[hb[int(ho[5 * t + j]):int(ho[5 * t + j + 1])].tobytes() for j in range(5)] for t in range(ntx)]
    ids_l, _ = engine.tx_ids(cash_leaves)
    cash_sigs = [[(ED,) + _sign(oracle, hashlib.sha256(b"tpl%d" % t).digest(), ids_l[t].tobytes())]
                 for t in range(ntx)]
    cash_sigs[17] = [(ED, cash_sigs[17][0][1], bytes(64))]
    tio = np.arange(0, 5 * ntx + 1, 5, dtype=np.uint64)

    def cash_call():
        res = engine.signed_txcomp_verify_arrays(blob, it, tio, cash_sigs)
        _compare(engine, cash_leaves, res, cash_sigs)
        assert res[1][17] == 1 and (res[1] == 0).sum() == ntx - 1

    for _ in range(3):  # the shapes built, then calls without misses: templates-only from here
        cash_call()
    r = random.Random(54)
    lens = r.sample(range(1500, 3000), 40)
    txs = [[("String", "".join(chr(97 + r.randrange(26)) for _ in range(n)), 0), ("int", r.randrange(2**31), 0)]
           for n in lens]
    txs[7].append(("String", "w" * 70_000, 0))
    leaves = [[K.leaf(k, v, c) for k, v, c in tx] for tx in txs]
    ids = [_oracle_id(oracle, lv) for lv in leaves]
    sigs = [[(ED,) + _sign(oracle, hashlib.sha256(b"new%d" % t).digest(), ids[t])] for t in range(len(txs))]
    for _ in range(2):  # misses (redone); then the full chain again (direct items every time)
        res = engine.signed_txcomp_verify(txs, sigs)
        assert [res[0][t].tobytes() for t in range(len(txs))] == ids
        assert (res[1] == 0).all()
        _compare(engine, leaves, res, sigs)
    for _ in range(3):
        cash_call()


def test_fused_template_hashes_every_kind(engine, oracle):
    """The templates-only chain hashes leaves straight from their templates (no leaf bytes):
    a batch of every kind -- RAW leaves of 0..200 bytes, strings, keys, parties, commands,
    cash states, boxed primitives -- run until its shapes are built (full chain), then again
    (templates-only): ids equal the oracle's over the restatement's leaves every time."""
    rng = random.Random(55)
    ref_keys = [bytes.fromhex(v["A"]) for v in TK._key_vectors()]
    # few distinct shapes (the table then holds them all: no direct items, so the later
    # calls run the templates-only chain)
    cash_pool = [TK._cash_state(rng, ref_keys) for _ in range(6)]
    party_pool = [TK._party(rng, ref_keys) for _ in range(6)]
    txs = []
    for t in range(300):
        comps = [("cash_state", rng.choice(cash_pool), 52), ("party", rng.choice(party_pool), 52),
                 ("issue_command", ("net.corda.contracts.asset.Cash$Commands$Issue", rng.randrange(-2**63, 2**63),
                                    [(45, rng.choice(ref_keys)) for _ in range(rng.randrange(1, 4))]), 10),
                 ("raw", bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 15, 16, 17, 55, 56, 63, 64, 200])))
                  if t % 97 else rng.randbytes(5000 if t % 2 else 70_000), 0),
                 ("ed25519_key", rng.choice(ref_keys), 45), ("int", rng.randrange(-2**31, 2**31), 0),
                 ("long", rng.randrange(-2**63, 2**63), 0), ("String", "tx%d" % (t % 7), 0),
                 ("kotlin_object", K.TRANSACTION_TYPE_GENERAL, 0)]
        rng.shuffle(comps)
        txs.append(comps[:rng.randrange(1, len(comps) + 1)])
    leaves = [[K.leaf(k, v, c) for k, v, c in tx] for tx in txs]
    ids = [_oracle_id(oracle, lv) for lv in leaves]
    sigs = [[(ED,) + _sign(oracle, hashlib.sha256(b"fth%d" % t).digest(), ids[t])] for t in range(len(txs))]
    for _ in range(4):
        res = engine.signed_txcomp_verify(txs, sigs)
        assert [res[0][t].tobytes() for t in range(len(txs))] == ids
        assert (res[1] == 0).all() and (res[3] == 0).all()


def test_concurrent_tickets_one_device(engine, oracle):
    """Consecutive signed-tx calls overlap on one device (two buffer sets, the enqueue
    token handed on once a call's last chunk is enqueued): two cordahip_txcomp_submit
    tickets and one cordahip_tx_submit ticket outstanding at once, each with its own
    signatures (different corruptions) and output arrays, in many signature chunks and id
    slices, the component calls before and after their shapes are built (full chain, then
    the templates-only chain). Every id, tx status, first_bad_sig and signature status
    equals the leaf path's run alone; the ids equal the oracle's on a sample."""
    rng = np.random.default_rng(56)
    ntx = 6000
    blob, items, _ = cash_issue_items(rng.integers(0, 256, (ntx, 32), dtype=np.uint8),
                                      rng.integers(0, 256, (ntx, 32), dtype=np.uint8), bytes(range(32)),
                                      rng.integers(1, 10**9, ntx), rng.integers(-2**63, 2**63 - 1, ntx))
    it = items.reshape(-1).copy()
    host_it = it.copy()
    host_it["data"] += np.uint64(blob.ctypes.data)
    hb, ho = _lib.kryo_encode_array(host_it)
    leaves = [[hb[int(ho[5 * t + j]):int(ho[5 * t + j + 1])].tobytes() for j in range(5)] for t in range(ntx)]
    ids_l, _ = engine.tx_ids(leaves)
    assert [ids_l[t].tobytes() for t in range(0, ntx, 1499)] == [_oracle_id(oracle, leaves[t])
                                                                 for t in range(0, ntx, 1499)]
    base = [[(ED,) + _sign(oracle, hashlib.sha256(b"cc%d-%d" % (t, q)).digest(), ids_l[t].tobytes())
             for q in range(1 + t % 3)] for t in range(ntx)]

    def corrupt(period, phase):
        out = []
        for t, per in enumerate(base):
            per = list(per)
            if t % period == phase:
                q = t % len(per)
                per[q] = (ED, per[q][1], per[q][2][:9] + bytes([per[q][2][9] ^ 2]) + per[q][2][10:])
            out.append(per)
        return out

    sig_sets = [corrupt(10, 3), corrupt(7, 2), corrupt(13, 5)]
    want = [engine.signed_tx_verify(leaves, s) for s in sig_sets]  # the leaf path, one call at a time
    tio = np.arange(0, 5 * ntx + 1, 5, dtype=np.uint64)
    old = os.environ.get("CORDAHIP_TX_SIG_CHUNK")
    os.environ["CORDAHIP_TX_SIG_CHUNK"] = "2048"  # ~6 chunks and id slices per call
    try:
        for rnd in range(3):  # round 0 may build shapes (full chain); later rounds: templates-only
            tks = [engine.signed_txcomp_verify_arrays(blob, it, tio, sig_sets[0], async_=True, pinned_out=rnd % 2 == 0),
                   engine.signed_tx_verify(leaves, sig_sets[2], async_=True),
                   engine.signed_txcomp_verify_arrays(blob, it, tio, sig_sets[1], async_=True)]
            got = [tk.wait() for tk in tks]
            for g, w in zip(got, [want[0], want[2], want[1]]):
                ids_c, st_c, fb_c, sst_c = g
                ids_w, st_w, fb_w, sst_w = w
                assert np.array_equal(st_c, st_w), rnd
                assert np.array_equal(fb_c, fb_w), rnd
                assert np.array_equal(sst_c, sst_w), rnd
                assert np.array_equal(ids_c, ids_w), rnd
                assert (st_c == 1).sum() > 0 and (st_c == 0).sum() > ntx // 2
    finally:
        if old is None:
            del os.environ["CORDAHIP_TX_SIG_CHUNK"]
        else:
            os.environ["CORDAHIP_TX_SIG_CHUNK"] = old


def _device_comp_call(engine, blob, items, tio, sigs, group=1):
    """cordahip_signed_txcomp_verify_ed25519_device over host arrays (copied to the GPU);
    sigs[t] = [(ED, key, sig), ...]. Returns (ids, tx_status, first_bad, sig_status) as numpy."""
    import torch
    dev = torch.device("cuda:0")
    n = len(tio) - 1
    flat = [x for per in sigs for x in per]
    so = np.zeros(n + 1, np.int64)
    so[1:] = np.cumsum([len(per) for per in sigs])
    d_items = torch.from_numpy(np.ascontiguousarray(items).view(np.uint8).copy()).to(dev)
    d_blob = torch.from_numpy(np.ascontiguousarray(blob, dtype=np.uint8).copy()).to(dev) if len(blob) else \
        torch.zeros(16, dtype=torch.uint8, device=dev)[:0]
    d_tio = torch.from_numpy(np.asarray(tio, np.int64)).to(dev)
    d_so = torch.from_numpy(so).to(dev)
    k = torch.from_numpy(np.frombuffer(b"".join(x[1] for x in flat) or bytes(32), np.uint8).reshape(-1, 32).copy()).to(dev)
    s = torch.from_numpy(np.frombuffer(b"".join(x[2] for x in flat) or bytes(64), np.uint8).reshape(-1, 64).copy()).to(dev)
    k, s = k[:len(flat)], s[:len(flat)]
    txid = torch.zeros((max(n, 1), 32), dtype=torch.uint8, device=dev)
    st = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
    fb = torch.zeros(max(n, 1), dtype=torch.int64, device=dev)
    sst = torch.zeros(max(len(flat), 1), dtype=torch.uint8, device=dev)
    engine.signed_txcomp_verify_ed25519_device(d_items, len(items), d_blob, d_tio, d_so, k, s, txid, st, fb, sst,
                                               group=group)
    torch.cuda.synchronize()
    return txid.cpu().numpy()[:n], st.cpu().numpy()[:n], fb.cpu().numpy()[:n], sst.cpu().numpy()[:len(flat)]


def _same(a, b, ctx=""):
    ids_a, st_a, fb_a, sst_a = a
    ids_b, st_b, fb_b, sst_b = b
    assert np.array_equal(st_a, st_b), ctx
    assert np.array_equal(fb_a, fb_b), ctx
    assert np.array_equal(sst_a, sst_b), ctx
    assert np.array_equal(ids_a[st_b == 0], ids_b[st_b == 0]), ctx


def test_device_component_call_every_kind(engine, oracle):
    """The device-resident component call (leaf hashes from the templates, new shapes traced
    in the same launch set, the rest through the direct encoder's SHA-256 sink) on random
    transactions of every kind -- invalid components, a transaction without components and
    ones without signatures, 70,000-character strings (no template: direct) -- called
    repeatedly (shapes built by the first call, hits afterwards): every output equals the
    host component path's, and the ids equal the oracle's over the restatement's leaves."""
    rng = random.Random(57)
    ntx = 300
    spec, comps = _random_txs(rng, ntx)
    comps[3], spec[3] = [], []
    for t in (11, 150):
        comps[t] = comps[t] + [("String", "d" * 70_000, 0)]
        spec[t] = spec[t] + [("String", "d" * 70_000, 0)]
    comps[40] = comps[40] + [("ed25519_key", b"k" * 31, 45)]  # rejected: BAD_COMPONENT
    leaves = [[K.leaf(k, v, c) for k, v, c in tx] for tx in spec]
    ids = [_oracle_id(oracle, lv) if lv and t != 40 else None for t, lv in enumerate(leaves)]
    sigs = _signers(oracle, rng, ids, ntx)
    host = engine.signed_txcomp_verify(comps, sigs)
    flat = [c for tx in comps for c in tx]
    blob, items, has = _lib.kryo_pack(flat)
    items = items.copy()
    items["data"] = np.where(has, items["data"], 0)
    tio = np.zeros(ntx + 1, np.uint64)
    tio[1:] = np.cumsum([len(tx) for tx in comps])
    for rnd in range(3):
        got = _device_comp_call(engine, blob, items, tio, sigs)
        _same(got, host, rnd)
        for t in range(ntx):
            if ids[t] is not None and sigs[t]:
                assert got[0][t].tobytes() == ids[t], (rnd, t)
        assert got[1][40] == _lib.TX_BAD_COMPONENT or not sigs[40]


def test_device_component_call_cash_corpus(engine, oracle):
    """The bench's cash-issue components through the device call (group = 5), corrupted
    signatures and components included, against the leaf path over the host encoder's leaves
    and the oracle's ids on a sample; a second corpus of other shapes between two calls."""
    rng = np.random.default_rng(58)
    ntx = 20000
    ik = rng.integers(0, 256, (ntx, 32), dtype=np.uint8)
    blob, items, layout = cash_issue_items(ik, rng.integers(0, 256, (ntx, 32), dtype=np.uint8), bytes(range(32)),
                                           rng.integers(1, 10**9, ntx), rng.integers(-2**63, 2**63 - 1, ntx))
    blob = blob.copy()
    for t in range(5, ntx, 1000):  # a flipped owner-key byte: another id, the signatures fail
        blob[layout["owner_key"] + t * layout["cash_stride"]] ^= 1
    it = items.reshape(-1).copy()
    host_it = it.copy()
    host_it["data"] += np.uint64(blob.ctypes.data)
    hb, ho = _lib.kryo_encode_array(host_it)
    leaves = [[hb[int(ho[5 * t + j]):int(ho[5 * t + j + 1])].tobytes() for j in range(5)] for t in range(ntx)]
    ids_l, _ = engine.tx_ids(leaves)
    assert [ids_l[t].tobytes() for t in range(0, ntx, 1999)] == [_oracle_id(oracle, leaves[t])
                                                                 for t in range(0, ntx, 1999)]
    sig_id = ids_l.copy()
    for t in range(5, ntx, 1000):
        sig_id[t] ^= 0xff  # signed over the id before the corruption (any other id)
    sigs = []
    for t in range(ntx):
        per = []
        for q in range(1 + t % 3):
            pub, sg = _sign(oracle, hashlib.sha256(b"dc%d-%d" % (t, q)).digest(), sig_id[t].tobytes())
            if t % 17 == 4 and q == 0:
                sg = sg[:20] + bytes([sg[20] ^ 8]) + sg[21:]
            per.append((ED, pub, sg))
        sigs.append(per)
    want = engine.signed_tx_verify(leaves, sigs)
    tio = np.arange(0, 5 * ntx + 1, 5, dtype=np.uint64)
    got = _device_comp_call(engine, blob, it, tio, sigs, group=5)
    _same(got, want)
    assert (want[1] == 1).sum() == len(set(range(5, ntx, 1000)) | set(range(4, ntx, 17)))
    other = [[("String", "x" * (100 + t), 0), ("long", t, 0)] for t in range(50)]
    ob, oi, oh = _lib.kryo_pack([c for tx in other for c in tx])
    oi = oi.copy()
    oi["data"] = np.where(oh, oi["data"], 0)
    oleaves = [[K.leaf(k, v, c) for k, v, c in tx] for tx in other]
    oids = [_oracle_id(oracle, lv) for lv in oleaves]
    osigs = [[(ED,) + _sign(oracle, b"\x21" * 32, oids[t])] for t in range(50)]
    og = _device_comp_call(engine, ob, oi, np.arange(0, 101, 2, dtype=np.uint64), osigs)
    assert [og[0][t].tobytes() for t in range(50)] == oids and (og[1] == 0).all()
    got = _device_comp_call(engine, blob, it, tio, sigs, group=5)
    _same(got, want)


def test_raw_leaf_over_2_29_bytes(engine, oracle):
    """A RAW component of 2^29 + 3 bytes (512 MiB): kryo_hash takes leaves under 2^29 bytes,
    so the templates-only chain counts it a miss (the call is redone with the full chain) and
    the device chain hashes it through the direct encoder's SHA-256 sink (64-bit bit length).
    Its transaction's id against hashlib (one leaf: the root is the leaf hash)."""
    big = np.frombuffer(np.random.default_rng(59).bytes((1 << 29) + 3), np.uint8)
    leaf_hash = hashlib.sha256(big.tobytes()).digest()
    items = np.zeros(1, _lib.KRYO_ITEM_DTYPE)
    items[0]["kind"], items[0]["len"], items[0]["data"] = 0, big.size, 0
    tio = np.array([0, 1], np.uint64)
    sigs = [[(ED,) + _sign(oracle, b"\x31" * 32, leaf_hash)]]
    # small component batches first, so the device's component calls run the templates-only chain
    small = [[("int", 7, 0), ("long", 9, 0)]] * 4
    sm_ids = [_oracle_id(oracle, [K.leaf(k, v, c) for k, v, c in tx]) for tx in small]
    for _ in range(3):
        engine.signed_txcomp_verify(small, [[(ED,) + _sign(oracle, b"\x32" * 32, i)] for i in sm_ids])
    print("templates-only chain warm; the 512 MiB leaf through the host call", flush=True)
    host = engine.signed_txcomp_verify_arrays(big, items, tio, sigs)
    assert host[0][0].tobytes() == leaf_hash and host[1][0] == 0 and host[3][0] == 0
    print("host call ok; the device call", flush=True)
    dev = _device_comp_call(engine, big, items, tio, sigs)
    assert dev[0][0].tobytes() == leaf_hash and dev[1][0] == 0 and dev[3][0] == 0
