"""CSR validation at the C-ABI on the GPU build (ABI 4): for every host entry
point that takes CSR arrays -- cordahip_sig_verify / _sig_submit,
cordahip_tx_ids / _txid_submit, cordahip_signed_tx_verify / _tx_submit,
cordahip_signed_txcomp_verify / _txcomp_submit, cordahip_filtered_tx_verify /
_filtered_tx_submit -- a batch with one bad offset (non-decreasing broken, or
past its declared buffer) or a short declared length returns
CORDAHIP_ERR_INVALID_ARG, never a crash; the same context then verifies the
corrected batch with the results of a fresh call (themselves checked against
the oracle in the other GPU tests; here the signatures against the C oracle).
The reference turns bad input into exceptions (Crypto.kt:472-483,
SignedTransaction.kt:37-39)."""
import ctypes
import hashlib

import numpy as np
import pytest

import kryo_leaves as K
from corda_amd import _lib
from corda_amd._lib import lib

pytestmark = pytest.mark.gpu
ED = 4
INVALID = -1


def _sign(oracle, seed, msg):
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    oracle.oracle_ed25519_sign(seed, msg, len(msg), pub, sig)
    return pub.raw, sig.raw


def _csr(items):
    off = np.zeros(len(items) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in items])
    blob = np.frombuffer(b"".join(items) or b"\0", np.uint8).copy()
    return blob, off


def _p(a):
    return a.ctypes.data


def _run(fn, batch, submit):
    """the call, synchronous or ticketed: its return code"""
    if not submit:
        return fn[0](engine_ctx(), ctypes.byref(batch))
    t = ctypes.c_uint64()
    rc = fn[1](engine_ctx(), ctypes.byref(batch), ctypes.byref(t))
    if rc != 0:
        return rc
    return lib().cordahip_wait(engine_ctx(), t.value, -1)


_ENG = []


def engine_ctx():
    return _ENG[0].ctx


@pytest.fixture(autouse=True)
def _ctx(engine):
    _ENG[:] = [engine]
    yield


@pytest.mark.parametrize("submit", [False, True])
def test_sig_batch_bad_offsets(engine, oracle, submit):
    n = 300
    msgs = [hashlib.sha256(b"csr%d" % i).digest() for i in range(n)]
    keys, sigs = zip(*[_sign(oracle, hashlib.sha256(b"k%d" % i).digest(), msgs[i]) for i in range(n)])
    sigs = list(sigs)
    sigs[7] = sigs[7][:10] + bytes([sigs[7][10] ^ 1]) + sigs[7][11:]
    kb, ko = _csr(list(keys))
    sb, so = _csr(sigs)
    mb, mo = _csr(msgs)
    sch = np.full(n, ED, np.uint8)
    st = np.zeros(n, np.uint8)
    vd = np.zeros((n + 63) // 64, np.uint64)
    fns = (lib().cordahip_sig_verify, lib().cordahip_sig_submit)

    def batch(ko_, so_, mo_, kbytes=kb.size, sbytes=sb.size, mbytes=mb.size):
        return _lib.SigBatch(n, _p(sch), _p(kb), _p(ko_), _p(sb), _p(so_), _p(mb), _p(mo_), _p(st), _p(vd), 0,
                             kbytes, sbytes, mbytes)

    bad = []
    k2 = ko.copy()
    k2[150] = k2[151] + 5  # not non-decreasing
    bad.append(batch(k2, so, mo))
    s2 = so.copy()
    s2[n] = sb.size + 64  # past the blob
    bad.append(batch(ko, s2, mo))
    m2 = mo.copy()
    m2[299] = 2 ** 64 - 1
    bad.append(batch(ko, so, m2))
    bad.append(batch(ko, so, mo, kbytes=kb.size - 1))  # a declared length short of the last key
    for b in bad:
        assert _run(fns, b, submit) == INVALID
    good = batch(ko, so, mo)
    assert _run(fns, good, submit) == 0
    want = np.zeros(n, np.uint8)
    M = np.frombuffer(b"".join(msgs), np.uint8).reshape(n, 32).copy()
    Kk = np.frombuffer(b"".join(keys), np.uint8).reshape(n, 32).copy()
    S = np.frombuffer(b"".join(sigs), np.uint8).reshape(n, 64).copy()
    oracle.oracle_ed25519_verify_batch(n, Kk.ctypes.data, S.ctypes.data, M.ctypes.data, 32, want.ctypes.data, 1)
    assert np.array_equal(st, want) and st[7] == 1 and (st == 0).sum() == n - 1


def _tx_arrays(oracle, ntx=200):
    txs = [[bytes([t % 251, q]) * (5 + q * 7) for q in range(1 + t % 5)] for t in range(ntx)]
    leaves = [x for tx in txs for x in tx]
    lb, lo = _csr(leaves)
    tlo = np.zeros(ntx + 1, np.uint64)
    tlo[1:] = np.cumsum([len(tx) for tx in txs])
    return txs, leaves, lb, lo, tlo


@pytest.mark.parametrize("submit", [False, True])
def test_tx_ids_bad_offsets(engine, oracle, submit):
    txs, leaves, lb, lo, tlo = _tx_arrays(oracle)
    ntx = len(txs)
    txid = np.zeros((ntx, 32), np.uint8)
    st = np.zeros(ntx, np.uint8)
    fns = (lib().cordahip_tx_ids, lib().cordahip_txid_submit)

    def batch(lo_, tlo_, nleaves=len(leaves), lbytes=lb.size):
        return _lib.TxidBatch(ntx, _p(lb), _p(lo_), _p(tlo_), _p(txid), _p(st), nleaves, lbytes)

    t2 = tlo.copy()
    t2[ntx] = len(leaves) + 1  # past nleaves
    l2 = lo.copy()
    l2[40], l2[41] = l2[41], l2[40] + 1  # out of order
    for b in (batch(lo, t2), batch(l2, tlo), batch(lo, tlo, lbytes=lb.size - 1), batch(lo, tlo, nleaves=3)):
        assert _run(fns, b, submit) == INVALID
    assert _run(fns, batch(lo, tlo), submit) == 0
    want, wst = engine.tx_ids(txs)
    assert np.array_equal(txid, want) and (st == wst).all()


def _sig_level(oracle, ids, ntx):
    per = [[(ED,) + _sign(oracle, hashlib.sha256(b"s%d-%d" % (t, q)).digest(), ids[t].tobytes())
            for q in range(1 + t % 3)] for t in range(ntx)]
    per[5] = [(ED, per[5][0][1], bytes(64))]  # a bad signature: first_bad 0
    flat = [x for p in per for x in p]
    tso = np.zeros(ntx + 1, np.uint64)
    tso[1:] = np.cumsum([len(p) for p in per])
    kb, ko = _csr([x[1] for x in flat])
    sb, so = _csr([x[2] for x in flat])
    return per, flat, tso, np.full(len(flat), ED, np.uint8), kb, ko, sb, so


@pytest.mark.parametrize("submit", [False, True])
def test_signed_tx_bad_offsets(engine, oracle, submit):
    txs, leaves, lb, lo, tlo = _tx_arrays(oracle)
    ntx = len(txs)
    ids, _ = engine.tx_ids(txs)
    per, flat, tso, sch, kb, ko, sb, so = _sig_level(oracle, ids, ntx)
    txid, st = np.zeros((ntx, 32), np.uint8), np.zeros(ntx, np.uint8)
    sst, fb = np.zeros(len(flat), np.uint8), np.zeros(ntx, np.int64)
    fns = (lib().cordahip_signed_tx_verify, lib().cordahip_tx_submit)

    def batch(tso_=tso, ko_=ko, so_=so, tlo_=tlo, nsig=len(flat), kbytes=kb.size):
        tb = _lib.TxidBatch(ntx, _p(lb), _p(lo), _p(tlo_), _p(txid), _p(st), len(leaves), lb.size)
        return _lib.SignedTxBatch(tb, _p(tso_), _p(sch), _p(kb), _p(ko_), _p(sb), _p(so_), _p(sst), _p(fb), nsig,
                                  kbytes, sb.size)

    a = tso.copy()
    a[100] = a[101] + 1
    b2 = ko.copy()
    b2[len(flat)] = kb.size + 32
    c = so.copy()
    c[3] = 0
    d = tlo.copy()
    d[0] = 5  # tx_leaf_off[0] > tx_leaf_off[1]
    for b in (batch(tso_=a), batch(ko_=b2), batch(so_=c), batch(tlo_=d), batch(nsig=len(flat) - 1),
              batch(kbytes=0)):
        assert _run(fns, b, submit) == INVALID
    assert _run(fns, batch(), submit) == 0
    w = engine.signed_tx_verify(txs, per)
    assert np.array_equal(txid, w[0]) and np.array_equal(st, w[1]) and np.array_equal(fb, w[2])
    assert np.array_equal(sst, w[3]) and st[5] == 1 and fb[5] == 0


@pytest.mark.parametrize("submit", [False, True])
def test_signed_txcomp_bad_offsets(engine, oracle, submit):
    comps = [[("int", t, 0), ("String", "tx-%d" % t, 0), ("long", -t, 0)][: 1 + t % 3] for t in range(120)]
    ntx = len(comps)
    leaves = [[K.leaf(k, v, c) for k, v, c in tx] for tx in comps]
    ids, _ = engine.tx_ids(leaves)
    per, flat, tso, sch, kb, ko, sb, so = _sig_level(oracle, ids, ntx)
    blob, items, has = _lib.kryo_pack([c for tx in comps for c in tx])
    items = items.copy()
    items["data"] = np.where(has, items["data"], 0)
    blob = np.ascontiguousarray(blob)
    tio = np.zeros(ntx + 1, np.uint64)
    tio[1:] = np.cumsum([len(tx) for tx in comps])
    txid, st = np.zeros((ntx, 32), np.uint8), np.zeros(ntx, np.uint8)
    sst, fb = np.zeros(len(flat), np.uint8), np.zeros(ntx, np.int64)
    fns = (lib().cordahip_signed_txcomp_verify, lib().cordahip_txcomp_submit)

    def batch(tio_=tio, n_items=len(items), tso_=tso, nsig=len(flat)):
        tb = _lib.TxcompBatch(ntx, _p(items), _p(tio_), _p(blob), blob.size, _p(txid), _p(st), n_items)
        return _lib.SignedTxcompBatch(tb, _p(tso_), _p(sch), _p(kb), _p(ko), _p(sb), _p(so), _p(sst), _p(fb), nsig,
                                      kb.size, sb.size)

    a = tio.copy()
    a[60] = a[61] + 2
    c = tso.copy()
    c[ntx] = len(flat) + 1
    for b in (batch(tio_=a), batch(n_items=len(items) - 1), batch(tso_=c), batch(nsig=0)):
        assert _run(fns, b, submit) == INVALID
    assert _run(fns, batch(), submit) == 0
    w = engine.signed_tx_verify(leaves, per)
    assert np.array_equal(txid, w[0]) and np.array_equal(st, w[1]) and np.array_equal(fb, w[2])
    assert np.array_equal(sst, w[3])


@pytest.mark.parametrize("submit", [False, True])
def test_filtered_tx_bad_offsets(engine, oracle, submit):
    import json
    import os
    cases = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                        "pmt_vectors.json")))["cases"]
    ftxs = [([bytes.fromhex(x) for x in c["leaves"]], [(t, bytes.fromhex(h) if h else None) for t, h in c["tokens"]],
             bytes.fromhex(c["root"])) for c in cases if c["leaves"] and c["tokens"]]
    want = engine.filtered_tx_verify(ftxs)
    leaves = [x for f in ftxs for x in f[0]]
    lb, lo = _csr(leaves)
    tlo = np.zeros(len(ftxs) + 1, np.uint64)
    tlo[1:] = np.cumsum([len(f[0]) for f in ftxs])
    toks = [t for f in ftxs for t in f[1]]
    tko = np.zeros(len(ftxs) + 1, np.uint64)
    tko[1:] = np.cumsum([len(f[1]) for f in ftxs])
    tok = np.array([t[0] for t in toks], np.uint8)
    th = np.frombuffer(b"".join((t[1] or bytes(32)) for t in toks), np.uint8).copy()
    root = np.frombuffer(b"".join(f[2] for f in ftxs), np.uint8).copy()
    st = np.zeros(len(ftxs), np.uint8)
    fns = (lib().cordahip_filtered_tx_verify, lib().cordahip_filtered_tx_submit)

    def batch(tlo_=tlo, lo_=lo, tko_=tko, ntok=len(toks)):
        return _lib.FilteredTxBatch(len(ftxs), _p(lb), _p(lo_), _p(tlo_), _p(tok), _p(th), _p(tko_), _p(root), _p(st),
                                    len(leaves), lb.size, ntok)

    a = tko.copy()
    a[10] = a[11] + 3
    c = lo.copy()
    c[len(leaves)] = lb.size + 1
    for b in (batch(tko_=a), batch(lo_=c), batch(ntok=len(toks) - 1)):
        assert _run(fns, b, submit) == INVALID
    assert _run(fns, batch(), submit) == 0
    assert np.array_equal(st, want) and (st == 0).sum() > 0
