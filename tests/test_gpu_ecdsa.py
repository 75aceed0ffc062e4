"""K2 parity on the GPU: secp256k1 / P-256 lanes vs the BouncyCastle-1.57 oracle,
through the C-ABI (generic CSR batch and the dense device path)."""
import hashlib
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_golden_vectors(engine, ec_vectors):
    st, verdict = engine.verify_batch([v["scheme"] for v in ec_vectors], [v["pub"] for v in ec_vectors],
                                      [v["sig"] for v in ec_vectors], [v["msg"] for v in ec_vectors])
    bad = [(v["cat"], v["scheme"], v["note"], int(s), v["status"]) for v, s in zip(ec_vectors, st)
           if s != v["status"]]
    assert not bad, bad[:20]


def test_mixed_with_ed25519_and_unsupported(engine, ec_vectors, ed_vectors):
    vs = ec_vectors[:200] + ed_vectors[:200]
    schemes = [v.get("scheme", 4) for v in vs] + [1, 5]
    keys = [v["pub"] for v in vs] + [b"k", b"k"]
    sigs = [v["sig"] for v in vs] + [b"s", b"s"]
    msgs = [v["msg"] for v in vs] + [b"m", b"m"]
    st, _ = engine.verify_batch(schemes, keys, sigs, msgs)
    assert [int(x) for x in st] == [v["status"] for v in vs] + [4, 4]


def _corpus(n, seed):
    import bc_ecdsa as ec
    rng = random.Random(seed)
    rows = []
    for i in range(n):
        scheme = 2 if i % 2 == 0 else 3
        c = ec.CURVES[scheme]
        d = rng.randrange(1, c.n)
        pub = ec.keypair(scheme, d)
        if i % 7 == 0:
            pub = ec.compress(pub)
        m = hashlib.sha256(b"tx%d-%d" % (seed, i)).digest()
        r, s = ec.sign(scheme, d, m, rng.randrange(1, c.n))
        if i % 3 == 0:
            s = c.n - s  # high-S: still valid
        sig = ec.der_encode(r, s)
        if i % 11 == 0:
            b = bytearray(sig)
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
            sig = bytes(b)
        rows.append((scheme, pub, sig, m))
    return rows


def test_random_vs_c_oracle(engine, oracle):
    rows = _corpus(600, 5)
    st, _ = engine.verify_batch(*zip(*rows))
    for (scheme, pub, sig, m), got in zip(rows, st):
        assert got == oracle.oracle_ecdsa_verify(scheme, pub, len(pub), sig, len(sig), m, len(m))
    assert (st == 0).sum() > 450


def test_device_path(engine, oracle):
    torch = pytest.importorskip("torch")
    rows = _corpus(512, 6)
    n = len(rows)
    keys = np.zeros((n, 65), np.uint8)
    sigs = np.zeros((n, 72), np.uint8)
    kl = np.zeros(n, np.uint8)
    sl = np.zeros(n, np.uint8)
    for i, (_, p, s, _) in enumerate(rows):
        keys[i, :len(p)] = np.frombuffer(p, np.uint8)
        kl[i] = len(p)
        sigs[i, :len(s)] = np.frombuffer(s, np.uint8)
        sl[i] = len(s)
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    sch = t(np.array([r[0] for r in rows], np.uint8))
    msgs = t(np.frombuffer(b"".join(r[3] for r in rows), np.uint8).reshape(n, 32))
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    verdict = torch.empty(n // 64, dtype=torch.int64, device=dev)
    engine.ecdsa_verify_device(sch, t(keys), t(kl), t(sigs), t(sl), msgs, status, verdict)
    torch.cuda.synchronize()
    got = status.cpu().numpy()
    want = [oracle.oracle_ecdsa_verify(r[0], r[1], len(r[1]), r[2], len(r[2]), r[3], 32) for r in rows]
    assert list(got) == want
    v = verdict.cpu().numpy().view(np.uint64)
    for i in range(n):
        assert ((int(v[i // 64]) >> (i % 64)) & 1) == (want[i] == 0)


def test_device_signer_matches_oracle(engine):
    """cordahip_ecdsa_sign_device (C3 corpus generator) vs the Python oracle, then
    its output through the device verifier."""
    import torch
    import bc_ecdsa as ec
    n, L = 192, 32
    rng = np.random.default_rng(9)
    scheme = np.where(rng.random(n) < 0.5, 2, 3).astype(np.uint8)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, L), dtype=np.uint8)
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(v).to(dev) for k, v in (("scheme", scheme), ("seeds", seeds), ("msgs", msgs))}
    keys = torch.zeros((n, 65), dtype=torch.uint8, device=dev)
    kl = torch.zeros(n, dtype=torch.uint8, device=dev)
    sigs = torch.zeros((n, 72), dtype=torch.uint8, device=dev)
    sl = torch.zeros(n, dtype=torch.uint8, device=dev)
    engine.ecdsa_sign_device(t["scheme"], t["seeds"], t["msgs"], keys, kl, sigs, sl)
    torch.cuda.synchronize()
    K, KL, S, SL = (x.cpu().numpy() for x in (keys, kl, sigs, sl))
    for i in range(n):
        c = ec.CURVES[int(scheme[i])]
        d = int.from_bytes(hashlib.sha256(seeds[i].tobytes()).digest(), "big") % c.n or 1
        k = int.from_bytes(hashlib.sha256(seeds[i].tobytes() + msgs[i].tobytes()).digest(), "big") % c.n or 1
        assert KL[i] == 65 and K[i].tobytes() == ec.keypair(int(scheme[i]), d), i
        want = ec.der_encode(*ec.sign(int(scheme[i]), d, msgs[i].tobytes(), k))
        assert S[i, :SL[i]].tobytes() == want, i
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    engine.ecdsa_verify_device(t["scheme"], keys, kl, sigs, sl, t["msgs"], st)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()


def _x_vector(ec, scheme, x_start, r_is_x, rng, tag):
    """A valid signature whose R = u1 G + u2 Q has x(R) >= x_start (key solved for)."""
    c = ec.CURVES[scheme]
    n, xr = c.n, x_start
    while True:
        rhs = (xr ** 3 + c.a * xr + c.b) % c.p
        yr = pow(rhs, (c.p + 1) // 4, c.p)
        if yr * yr % c.p == rhs:
            break
        xr += 1
    r = xr if r_is_x else xr - n
    m = hashlib.sha256(b"xcheck-%d" % tag).digest()
    e = int.from_bytes(hashlib.sha256(m).digest(), "big")
    s = rng.randrange(1, n)
    w = pow(s, n - 2, n)
    u1, u2 = e * w % n, r * w % n
    Q = ec._mul(c, pow(u2, n - 2, n), ec._add(c, (xr, yr), ec._mul(c, n - u1, c.G)))
    pub = b"\x04" + Q[0].to_bytes(32, "big") + Q[1].to_bytes(32, "big")
    return scheme, pub, ec.der_encode(r, s), m


def test_x_coordinate_check_ranges(engine):
    """The inversion-free x(P) mod n == r check on both of its branches: x(P) < n
    (X == r Z^2) and x(P) in [n, p) (X == (r + n) Z^2), with x near n, near p and
    at 2^255, on both curves, against the oracle."""
    import bc_ecdsa as ec
    rng = random.Random(33)
    rows = []
    for scheme in (2, 3):
        c = ec.CURVES[scheme]
        for start, r_is_x in ((c.n + 1, False), (c.n - 2**20, True), (c.p - 2**40, False), (2**255, True),
                              (c.n + 2**100, False), (c.n + 2**100, True)):
            rows.append(_x_vector(ec, scheme, start, r_is_x, rng, len(rows)))
    st, _ = engine.verify_batch(*zip(*rows))
    want = [ec.verify_status(*r) for r in rows]
    assert [int(x) for x in st] == want
    assert want.count(0) == 10  # the two r = x(P) >= n rows are range-rejected


def test_batch_inversion_boundaries(engine, ec_vectors):
    """The split path inverts s in runs of 16 slots per thread (Montgomery's
    trick) over the curve-partitioned order: odd batch sizes, runs that straddle
    the secp256k1 / P-256 boundary and runs full of already-decided lanes must
    all give the golden statuses."""
    rng = random.Random(21)
    for n in (1, 2, 15, 16, 17, 31, 33, 63, 65, 130, 257):
        vs = [ec_vectors[rng.randrange(len(ec_vectors))] for _ in range(n)]
        st, _ = engine.verify_batch([v["scheme"] for v in vs], [v["pub"] for v in vs], [v["sig"] for v in vs],
                                    [v["msg"] for v in vs])
        assert [int(x) for x in st] == [v["status"] for v in vs], n


def test_message_lengths_and_alignments(engine, oracle):
    """e = SHA-256(clear data) for every length 0..140 (and 200, 1000) at every
    byte alignment of the CSR blob (Crypto.doVerify takes any clearData; the
    reference only ever passes 32-byte ids, so this pins the generic path):
    valid signatures verify, a flipped message bit rejects, empty -> EMPTY."""
    import bc_ecdsa as bc
    rng = random.Random(33)
    schemes, keys, sigs, msgs = [], [], [], []
    for ln in list(range(141)) + [200, 1000]:
        sch = 2 + (ln & 1)
        d = rng.randrange(1, 1 << 250)
        pub = bc.keypair(sch, d)
        msg = bytes(rng.getrandbits(8) for _ in range(ln))
        r, s = bc.sign(sch, d, msg, rng.randrange(1, 1 << 250))
        sig = bc.der_encode(r, s)
        if ln % 3 == 2:
            msg = msg[:-1] + bytes([msg[-1] ^ 0x10])
        schemes.append(sch)
        keys.append(pub if ln % 4 else bc.compress(pub))
        sigs.append(sig)
        msgs.append(msg)
    st, _ = engine.verify_batch(schemes, keys, sigs, msgs)
    for i, (sch, k, g, m) in enumerate(zip(schemes, keys, sigs, msgs)):
        want = oracle.oracle_ecdsa_verify(sch, k, len(k), g, len(g), m, len(m))
        assert st[i] == want, (i, len(m), st[i], want)
        assert want == (5 if not m else 1 if len(m) % 3 == 2 else 0)


def test_reference_certificate_signatures(engine, cert_vectors):
    """K2 against signatures made by the reference's own BouncyCastle path (the
    ecdsa-with-SHA256 certificates shipped in /root/reference, both curves; 430-510
    byte TBS messages, so the multi-block SHA-256 path too) and their derived
    corruptions, through the generic C-ABI batch and the dense device path."""
    vs = cert_vectors
    st, verdict = engine.verify_batch([v["scheme"] for v in vs], [v["pub"] for v in vs], [v["sig"] for v in vs],
                                      [v["msg"] for v in vs])
    bad = [(v["cat"], v["cert"], int(s), v["status"]) for v, s in zip(vs, st) if s != v["status"]]
    assert not bad, bad
    for i, v in enumerate(vs):
        assert ((int(verdict[i // 64]) >> (i % 64)) & 1) == (v["status"] == 0)
