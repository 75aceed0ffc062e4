"""The device-memory budget and the idle release (ABI 4: CORDAHIP_DEVICE_MEM_BUDGET,
cordahip_device_mem, cordahip_trim, CORDAHIP_IDLE_RELEASE_MS) on the GPU: a context
with a 64 MiB budget sizes its Ed25519 workspace at ~9.4 k lanes and its ECDSA
workspace at ~9 k slots, so C2-, C3- and c4h-shaped batches run in several launch
sets each; every result matches the construction and the C oracle on samples; the
bytes the library holds stay within the budget's workspaces plus the batch
buffers; cordahip_trim and the idle release give them back, and the context
verifies again afterwards. (Host process reference: the JVM node that hosts the
library, SignedTransaction.kt:95-100.)"""
import ctypes
import hashlib
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ED = 4
MIB = 1 << 20


@pytest.fixture(scope="module")
def small():
    import torch  # noqa: F401
    from corda_amd.engine import Engine
    old = {k: os.environ.get(k) for k in ("CORDAHIP_DEVICE_MEM_BUDGET", "CORDAHIP_IDLE_RELEASE_MS")}
    os.environ["CORDAHIP_DEVICE_MEM_BUDGET"] = "64M"
    os.environ["CORDAHIP_IDLE_RELEASE_MS"] = "400"
    try:
        eng = Engine(1)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    yield eng
    eng.close()


def test_budget_reported(small):
    in_use, peak, budget = small.device_mem(0)
    assert budget == 64 * MIB and peak >= in_use > 0


def test_c2_shape_in_several_launch_sets(small, oracle):
    import torch
    from corda_amd.corpus import make_c2_corpus
    dev = torch.device("cuda:0")
    n = 50_000  # > 9,408 lanes of workspace: 6 launch pairs
    pubs, sigs, msgs, exp, _ = make_c2_corpus(small, n, 0xC0DA0601, dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    base = small.device_mem(0)[0]
    small.ed25519_verify_device(pubs, sigs, msgs, st, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = st.cpu()
    known = exp.cpu() >= 0
    assert (got[known].to(torch.int16) == exp.cpu()[known]).all()
    k = np.ascontiguousarray(pubs[:4000].cpu().numpy())
    s = np.ascontiguousarray(sigs[:4000].cpu().numpy())
    m = np.ascontiguousarray(msgs[:4000].cpu().numpy())
    want = np.zeros(4000, np.uint8)
    oracle.oracle_ed25519_verify_batch(4000, k.ctypes.data, s.ctypes.data, m.ctypes.data, 32, want.ctypes.data, 4)
    assert np.array_equal(got[:4000].numpy(), want)
    in_use, peak, budget = small.device_mem(0)
    # the workspace the budget allows (45% of it), nothing batch-sized on the device path
    assert in_use - base <= budget * 45 // 100 + MIB


def test_c3_shape_in_several_launch_sets(small, oracle):
    import torch
    from corda_amd.corpus import make_c3_corpus
    dev = torch.device("cuda:0")
    n = 30_000  # > ~9 k ECDSA slots: 4 launch sets
    scheme, keys, key_len, sigs, sig_len, msgs, exp, _ = make_c3_corpus(small, n, 0xC0DA0602, dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    small.ecdsa_verify_device(scheme, keys, key_len, sigs, sig_len, msgs, st, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = st.cpu()
    known = exp.cpu() >= 0
    assert (got[known].to(torch.int16) == exp.cpu()[known]).all()
    idx = np.arange(0, n, 15)
    sch, K, KL, S, SL, M = (x.cpu().numpy()[idx] for x in (scheme, keys, key_len, sigs, sig_len, msgs))
    kb = np.ascontiguousarray(np.concatenate([K[i, :KL[i]] for i in range(len(idx))]))
    sb = np.ascontiguousarray(np.concatenate([S[i, :SL[i]] for i in range(len(idx))]))
    ko = np.zeros(len(idx) + 1, np.uint64)
    so = np.zeros(len(idx) + 1, np.uint64)
    ko[1:] = np.cumsum(KL.astype(np.uint64))
    so[1:] = np.cumsum(SL.astype(np.uint64))
    mo = np.arange(len(idx) + 1, dtype=np.uint64) * 32
    want = np.zeros(len(idx), np.uint8)
    Mc = np.ascontiguousarray(M)
    sch = np.ascontiguousarray(sch)
    oracle.oracle_ecdsa_verify_batch(len(idx), sch.ctypes.data, kb.ctypes.data, ko.ctypes.data, sb.ctypes.data,
                                     so.ctypes.data, Mc.ctypes.data, mo.ctypes.data, want.ctypes.data, 4)
    assert np.array_equal(got.numpy()[idx], want)


def _sign(oracle, seed, msg):
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    oracle.oracle_ed25519_sign(seed, msg, len(msg), pub, sig)
    return pub.raw, sig.raw


def test_c4h_shape_trim_and_idle_release(small, engine, oracle):
    ntx = 12_000
    txs = [[bytes([t % 256, q]) * (40 + 30 * q) for q in range(5)] for t in range(ntx)]
    ids, _ = engine.tx_ids(txs)
    sigs = []
    for t in range(ntx):
        per = [(ED,) + _sign(oracle, hashlib.sha256(b"m%d-%d" % (t, q)).digest(), ids[t].tobytes())
               for q in range(1 + t % 3)]
        if t % 11 == 4:
            per[-1] = (ED, per[-1][1], per[-1][2][:30] + bytes([per[-1][2][30] ^ 1]) + per[-1][2][31:])
        sigs.append(per)
    want = engine.signed_tx_verify(txs, sigs)  # the session context, default budget
    got = small.signed_tx_verify(txs, sigs)    # 64 MiB: every chunk in several launch pairs
    for a, b in zip(got, want):
        assert np.array_equal(a, b)
    assert (got[1] == 1).sum() == len(range(4, ntx, 11))
    before = small.device_mem(0)[0]
    small.trim()
    after = small.device_mem(0)[0]
    assert after < before
    # the idle release (400 ms here) after another call: the buffers go back by themselves
    got2 = small.signed_tx_verify(txs, sigs)
    assert all(np.array_equal(a, b) for a, b in zip(got2, want))
    grown = small.device_mem(0)[0]
    deadline = time.time() + 10
    while time.time() < deadline and small.device_mem(0)[0] >= grown:
        time.sleep(0.2)
    assert small.device_mem(0)[0] < grown
    got3 = small.signed_tx_verify(txs[:100], sigs[:100])  # and the context still verifies
    assert np.array_equal(got3[1], want[1][:100])


def test_component_slices_in_pieces(small, engine, oracle):
    """cordahip_txcomp_submit under the 64 MiB budget: the full encoder chain's leaf buffer
    is capped at a tenth of the budget (6.7 MB, ~300 cash-issue transactions' bound), so
    each id slice is encoded and hashed in pieces of whole transactions; ids, statuses and
    first_bad_sig equal the default context's and the oracle's ids"""
    from corda_amd import _lib
    from corda_amd.corpus import cash_issue_items
    rng = np.random.default_rng(61)
    ntx = 3000
    blob, items, _ = cash_issue_items(rng.integers(0, 256, (ntx, 32), dtype=np.uint8),
                                      rng.integers(0, 256, (ntx, 32), dtype=np.uint8), bytes(range(32)),
                                      rng.integers(1, 10**9, ntx), rng.integers(-2**63, 2**63 - 1, ntx))
    it = items.reshape(-1).copy()
    host_it = it.copy()
    host_it["data"] += np.uint64(blob.ctypes.data)
    hb, ho = _lib.kryo_encode_array(host_it)
    leaves = [[hb[int(ho[5 * t + j]):int(ho[5 * t + j + 1])].tobytes() for j in range(5)] for t in range(ntx)]
    ids_l, _ = engine.tx_ids(leaves)
    for t in range(0, ntx, 499):  # the oracle's ids on a sample
        want = ctypes.create_string_buffer(32)
        lb = np.frombuffer(b"".join(leaves[t]), np.uint8).copy()
        lo = np.zeros(6, np.uint64)
        lo[1:] = np.cumsum([len(x) for x in leaves[t]])
        assert oracle.oracle_tx_id(lb.ctypes.data, lo.ctypes.data, 5, want) == 0
        assert want.raw == ids_l[t].tobytes()
    sigs = []
    for t in range(ntx):
        pub, sg = _sign(oracle, hashlib.sha256(b"pc%d" % t).digest(), ids_l[t].tobytes())
        if t % 13 == 5:
            sg = sg[:7] + bytes([sg[7] ^ 2]) + sg[8:]
        sigs.append([(ED, pub, sg)] * (1 + t % 3))
    tio = np.arange(0, 5 * ntx + 1, 5, dtype=np.uint64)
    want = engine.signed_txcomp_verify_arrays(blob, it, tio, sigs)
    for _ in range(2):  # the first call on the small context runs the full chain
        got = small.signed_txcomp_verify_arrays(blob, it, tio, sigs)
        for a, b in zip(got, want):
            assert np.array_equal(a, b)
    assert np.array_equal(got[0][:ntx], ids_l[:ntx])
    assert (got[1] == 1).sum() == len(range(5, ntx, 13))
