"""The host-batch pipeline behind cordahip_sig_verify / cordahip_sig_submit (the
Crypto.isValid / doVerify batch, host_batch.cpp) on adversarial CSR batches:
every scheme byte, Ed25519 messages of many lengths (so a chunk holds several
length groups, each its own launch at a 16-B aligned message offset), ECDSA
lanes of both curves with messages of many lengths and DER signatures longer
than the 72-byte slot, wrong key and signature lengths, unsupported schemes,
interleaved at random. Statuses must equal the C oracle's (doVerify and
isValid semantics), in-process with the default chunking and in a subprocess
with 256-lane chunks (every chunk mixes groups and both sections; all three
pipeline stages reused many times)."""
import ctypes
import hashlib
import json
import os
import random
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def make_batch(oracle, n=2600, seed=5):
    import bc_ecdsa as ec
    rng = random.Random(seed)
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    lens = [0, 1, 31, 32, 33, 64, 100, 137]
    rows = []
    pool = {}  # per curve: (key, message, DER signature) made once (pure-Python signing is slow)
    for sch in (2, 3):
        c = ec.CURVES[sch]
        pool[sch] = []
        for j, ln in enumerate(lens * 3):
            d = rng.randrange(1, c.n)
            m = bytes(rng.getrandbits(8) for _ in range(ln))
            rr, ss = ec.sign(sch, d, m, rng.randrange(1, c.n))
            pool[sch].append((ec.keypair(sch, d), m, rr, ss))
    for i in range(n):
        kind = rng.random()
        msg = bytes(rng.getrandbits(8) for _ in range(rng.choice(lens)))
        if kind < 0.6:  # Ed25519
            oracle.oracle_ed25519_sign(hashlib.sha256(b"hb%d" % (i % 50)).digest(), msg, len(msg), pub, sig)
            k, s = pub.raw, bytearray(sig.raw)
            r = rng.random()
            if r < 0.1:
                s[rng.randrange(64)] ^= 1 << rng.randrange(8)
            elif r < 0.13:
                s = s[:rng.choice([0, 63])] if rng.random() < 0.5 else s + b"\x00"
            elif r < 0.15:
                k = k[:31]
            rows.append((4, k, bytes(s), msg))
        elif kind < 0.95:  # ECDSA, both curves
            sch = rng.choice((2, 3))
            pk, msg, rr, ss = pool[sch][rng.randrange(len(pool[sch]))]
            s = ec.der_encode(rr, ss)
            r = rng.random()
            if r < 0.1:
                b = bytearray(s)
                b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
                s = bytes(b)
            elif r < 0.14:  # longer than the slot: well-formed INTEGERs >= n, or garbage
                big = rng.getrandbits(8 * 40) | (1 << 319)
                s = ec.der_encode(big, ss) if rng.random() < 0.5 else bytes(rng.getrandbits(8) for _ in range(80))
            elif r < 0.16:
                s = b""
            key = ec.compress(pk) if rng.random() < 0.3 else pk
            if rng.random() < 0.03:
                key = key[:-1]
            rows.append((sch, key, s, msg))
        else:  # schemes the GPU does not take
            rows.append((rng.choice((0, 1, 5, 9)), bytes(32), bytes(64), msg))
    return rows


def oracle_status(oracle, rows, is_valid):
    out = []
    for sch, k, s, m in rows:
        if sch == 4:
            f = oracle.oracle_ed25519_is_valid if is_valid else oracle.oracle_ed25519_verify
            out.append(f(k, len(k), s, len(s), m, len(m)))
        elif sch in (2, 3):
            f = oracle.oracle_ecdsa_is_valid if is_valid else oracle.oracle_ecdsa_verify
            out.append(f(sch, k, len(k), s, len(s), m, len(m)))
        else:
            out.append(4)  # Crypto.kt:474: unsupported scheme
    return out


@pytest.mark.parametrize("is_valid", [False, True])
def test_host_batch_adversarial_vs_oracle(engine, oracle, is_valid):
    rows = make_batch(oracle)
    want = oracle_status(oracle, rows, is_valid)
    st, vd = engine.verify_batch(*zip(*rows), is_valid=is_valid)
    bad = [(i, rows[i][0], len(rows[i][1]), len(rows[i][2]), len(rows[i][3]), int(s), w)
           for i, (s, w) in enumerate(zip(st, want)) if int(s) != w]
    assert not bad, bad[:12]
    for i, w in enumerate(want):
        assert ((int(vd[i // 64]) >> (i % 64)) & 1) == (w == 0)


SCRIPT = r"""
import json, sys
sys.path.insert(0, %(root)r); sys.path.insert(0, %(root)r + "/tests"); sys.path.insert(0, %(root)r + "/oracle")
from conftest import load_oracle
from corda_amd.engine import Engine
from test_gpu_host_batch import make_batch, oracle_status
orc = load_oracle()
rows = make_batch(orc, n=3001, seed=9)
rows2 = make_batch(orc, n=2500, seed=10)
want = oracle_status(orc, rows, False)
want2 = oracle_status(orc, rows2, False)
with Engine(1) as eng:
    st, _ = eng.verify_batch(*zip(*rows))
    # the ticketed form, three calls outstanding at once (two transaction sets per
    # device: the third waits for a set; chunks of the first two interleave)
    tks = [eng.verify_batch(*zip(*r), async_=True) for r in (rows, rows2, rows)]
    st2, st3, st4 = (t.wait()[0] for t in tks)
bad = [i for i, (a, b, c, w) in enumerate(zip(st, st2, st4, want)) if int(a) != w or int(b) != w or int(c) != w]
bad += [("b2", i) for i, (a, w) in enumerate(zip(st3, want2)) if int(a) != w]
print(json.dumps({"n": len(rows), "bad": bad[:10]}))
sys.exit(1 if bad else 0)
"""


def test_host_batch_small_chunks_subprocess():
    env = dict(os.environ, CORDAHIP_HOST_CHUNK="256")
    r = subprocess.run([sys.executable, "-c", SCRIPT % {"root": ROOT}], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n"] == 3001


def test_host_batch_many_message_lengths(engine, oracle):
    """~300 distinct Ed25519 message lengths in one piece (the grouping's hash-map
    path, ADVICE r03: linear in the lanes however varied the lengths) plus runs of
    equal lengths (the previous-lane shortcut), every status against the oracle."""
    rng = random.Random(77)
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    rows = []
    for i in range(3000):
        ln = rng.randrange(0, 301) if i % 3 else 48 + (i // 300)
        msg = bytes(rng.getrandbits(8) for _ in range(ln))
        oracle.oracle_ed25519_sign(hashlib.sha256(b"ml%d" % (i % 40)).digest(), msg, len(msg), pub, sig)
        s = bytearray(sig.raw)
        if rng.random() < 0.1:
            s[rng.randrange(64)] ^= 1 << rng.randrange(8)
        rows.append((4, pub.raw, bytes(s), msg))
    want = oracle_status(oracle, rows, False)
    st, vd = engine.verify_batch(*zip(*rows))
    assert [int(x) for x in st] == want
    assert len({len(r[3]) for r in rows}) > 250


def test_bench_verdict_packing_matches_library(engine, oracle):
    """bench.py's C5 verdict words (statuses -> int64 words on the GPU, the operand
    of the N > 1 all-gather) equal the verdict words the library's own kernels
    build by wave ballot for the same statuses."""
    import torch
    sys.path.insert(0, ROOT)
    from bench import _pack_verdict
    n = 4096
    rng = random.Random(3)
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    k, s, m = bytearray(), bytearray(), bytearray()
    for i in range(n):
        msg = hashlib.sha256(b"pv%d" % i).digest()
        oracle.oracle_ed25519_sign(hashlib.sha256(b"pvk%d" % (i % 16)).digest(), msg, 32, pub, sig)
        b = bytearray(sig.raw)
        if rng.random() < 0.2:
            b[rng.randrange(64)] ^= 1
        k += pub.raw
        s += b
        m += msg
    dev = torch.device("cuda:0")
    tk, ts, tm = (torch.frombuffer(bytes(x), dtype=torch.uint8).view(n, -1).to(dev) for x in (k, s, m))
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    vd = torch.empty(n // 64, dtype=torch.int64, device=dev)
    engine.ed25519_verify_device(tk, ts, tm, st, vd, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert torch.equal(_pack_verdict(st), vd)
    assert 0 < int((st != 0).sum()) < n
