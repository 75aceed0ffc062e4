"""K1 parity on the GPU: libcordahip's Ed25519 lanes vs the i2p-0.2.0 oracle.

Every test calls the product through the C-ABI (ctypes -> libcordahip.so)
and compares bit-for-bit (status bytes and verdict words) with the golden
fixture (tests/golden/ed25519_vectors.json) or with oracle/c on seeded inputs.
"""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ED = 4


def test_golden_vectors_generic_batch(engine, ed_vectors):
    st, verdict = engine.verify_batch([ED] * len(ed_vectors), [v["pub"] for v in ed_vectors],
                                      [v["sig"] for v in ed_vectors], [v["msg"] for v in ed_vectors])
    bad = [(v["cat"], v["note"], int(s), v["status"]) for v, s in zip(ed_vectors, st) if s != v["status"]]
    assert not bad, bad[:20]
    for i, v in enumerate(ed_vectors):
        assert ((int(verdict[i // 64]) >> (i % 64)) & 1) == (v["status"] == 0)


def test_golden_vectors_dense_host(engine, ed_vectors):
    vs = [v for v in ed_vectors if len(v["pub"]) == 32 and len(v["sig"]) == 64 and len(v["msg"]) == 32]
    keys = np.frombuffer(b"".join(v["pub"] for v in vs), np.uint8)
    sigs = np.frombuffer(b"".join(v["sig"] for v in vs), np.uint8)
    msgs = np.frombuffer(b"".join(v["msg"] for v in vs), np.uint8)
    st, _ = engine.ed25519_verify_host(keys, sigs, msgs)
    assert [int(s) for s in st] == [v["status"] for v in vs]


def _corpus(oracle, n, seed):
    import ctypes
    keys = bytearray(32 * n)
    sigs = bytearray(64 * n)
    msgs = bytearray()
    pub = ctypes.create_string_buffer(32)
    sig = ctypes.create_string_buffer(64)
    for i in range(n):
        sd = hashlib.sha256(b"t%d-%d" % (seed, i)).digest()
        m = hashlib.sha256(b"m%d-%d" % (seed, i)).digest()
        oracle.oracle_ed25519_sign(sd, m, 32, pub, sig)
        keys[32 * i:32 * i + 32] = pub.raw
        sigs[64 * i:64 * i + 64] = sig.raw
        msgs += m
    return (np.frombuffer(bytes(keys), np.uint8).copy(), np.frombuffer(bytes(sigs), np.uint8).copy(),
            np.frombuffer(bytes(msgs), np.uint8).copy())


def _oracle_status(oracle, keys, sigs, msgs, n):
    out = np.zeros(n, np.uint8)
    oracle.oracle_ed25519_verify_batch(n, keys.ctypes.data, sigs.ctypes.data, msgs.ctypes.data, 32,
                                       out.ctypes.data, 8)
    return out


def test_random_corruption_vs_oracle(engine, oracle):
    n = 4096
    keys, sigs, msgs = _corpus(oracle, n, 1)
    rng = np.random.default_rng(7)
    sigs = sigs.reshape(n, 64)
    keys = keys.reshape(n, 32)
    for i in rng.choice(n, n // 4, replace=False):
        kind = i % 4
        if kind == 0:
            b = rng.integers(0, 512)
            sigs[i, b // 8] ^= 1 << (b % 8)
        elif kind == 1:
            keys[i, rng.integers(0, 32)] ^= 1 << rng.integers(0, 8)
        elif kind == 2:
            sigs[i, 63] |= 0x80  # S >= 2^255: exercises slide() carry drop
        else:
            sigs[i, 32:] = rng.integers(0, 256, 32, dtype=np.uint8)
    want = _oracle_status(oracle, keys, sigs, msgs, n)
    got, verdict = engine.ed25519_verify_host(keys, sigs, msgs)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:20]
    assert (want == 0).sum() > n // 2


def test_device_path_and_signer(engine, oracle):
    torch = pytest.importorskip("torch")
    n = 2048
    dev = torch.device("cuda:0")
    seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=dev)
    msgs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=dev)
    pubs = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sigs = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    engine.ed25519_sign_device(seeds, msgs, pubs, sigs)
    torch.cuda.synchronize()
    # GPU signer vs oracle signer (RFC 8032 is deterministic)
    import ctypes
    pub = ctypes.create_string_buffer(32)
    sg = ctypes.create_string_buffer(64)
    s_np, m_np, p_np, g_np = (t.cpu().numpy() for t in (seeds, msgs, pubs, sigs))
    for i in range(0, n, 97):
        oracle.oracle_ed25519_sign(s_np[i].tobytes(), m_np[i].tobytes(), 32, pub, sg)
        assert p_np[i].tobytes() == pub.raw and g_np[i].tobytes() == sg.raw, i
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    verdict = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
    engine.ed25519_verify_device(pubs, sigs, msgs, status, verdict)
    torch.cuda.synchronize()
    assert int(status.sum()) == 0
    assert bool((verdict == -1).all())


def test_reference_made_keys(engine, oracle):
    """The two Ed25519 keys the reference itself serialised (samples/irs-demo/
    .../trade.json:3,25, tests/golden/kryo_key_vectors.json): A5 decode succeeds
    on the GPU, so every arbitrary signature is BAD_SIG (not BAD_KEY), as in the
    oracle, through the generic batch, the dense host path and the device path."""
    import json
    import os
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    vs = json.load(open(os.path.join(root, "tests", "golden", "kryo_key_vectors.json")))["vectors"]
    rows = [(bytes.fromhex(v["A"]), bytes.fromhex(s["sig"]), bytes.fromhex(s["msg"]), s["status"])
            for v in vs for s in v["signatures"]]
    # each key also with 60 more arbitrary signatures
    for v in vs:
        for j in range(60):
            sig = hashlib.sha512(b"more%d" % j + bytes.fromhex(v["A"])).digest()
            msg = hashlib.sha256(b"msg%d" % j).digest()
            rows.append((bytes.fromhex(v["A"]), sig, msg, None))
    n = len(rows)
    keys = np.frombuffer(b"".join(r[0] for r in rows), np.uint8).copy()
    sigs = np.frombuffer(b"".join(r[1] for r in rows), np.uint8).copy()
    msgs = np.frombuffer(b"".join(r[2] for r in rows), np.uint8).copy()
    want = _oracle_status(oracle, keys, sigs, msgs, n)
    assert (want == 1).all()
    assert [int(w) for w, r in zip(want, rows) if r[3] is not None] == [r[3] for r in rows if r[3] is not None]
    st, _ = engine.verify_batch([ED] * n, [r[0] for r in rows], [r[1] for r in rows], [r[2] for r in rows])
    assert np.array_equal(st, want)
    st2, _ = engine.ed25519_verify_host(keys, sigs, msgs)
    assert np.array_equal(st2, want)
    dev = torch.device("cuda:0")
    tk, ts, tm = (torch.from_numpy(x.reshape(n, -1)).to(dev) for x in (keys, sigs, msgs))
    st3 = torch.empty(n, dtype=torch.uint8, device=dev)
    engine.ed25519_verify_device(tk, ts, tm, st3, None, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert np.array_equal(st3.cpu().numpy(), want)
