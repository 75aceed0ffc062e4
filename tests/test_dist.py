"""N > 1 path on CPU: world_size-2 gloo, exercising the same sharding and
verdict all-gather code bench.py uses over RCCL (corda_amd/dist.py). The
per-rank verification is the oracle here (no GPU in this container); the
test checks that sharding + gather reassemble the exact global verdict mask."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from corda_amd.dist import gather_verdicts, max_over_ranks, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _corpus(n):
    import conftest
    orc = conftest.load_oracle()
    import ctypes
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    k = np.zeros((n, 32), np.uint8)
    s = np.zeros((n, 64), np.uint8)
    m = np.zeros((n, 32), np.uint8)
    for i in range(n):
        msg = hashlib.sha256(b"dist%d" % i).digest()
        orc.oracle_ed25519_sign(hashlib.sha256(b"dseed%d" % i).digest(), msg, 32, pub, sig)
        k[i] = np.frombuffer(pub.raw, np.uint8)
        s[i] = np.frombuffer(sig.raw, np.uint8)
        m[i] = np.frombuffer(msg, np.uint8)
        if i % 3 == 0:
            s[i, 5] ^= 1
    return orc, k, s, m


def _verdict_words(orc, k, s, m, lo, hi, words):
    n = hi - lo
    st = np.zeros(max(n, 1), np.uint8)
    if n:
        kk, ss, mm = (np.ascontiguousarray(x[lo:hi]) for x in (k, s, m))
        orc.oracle_ed25519_verify_batch(n, kk.ctypes.data, ss.ctypes.data, mm.ctypes.data, 32, st.ctypes.data, 1)
    out = np.zeros(words, np.uint64)
    for j in range(n):
        if st[j] == 0:
            out[j // 64] |= np.uint64(1) << np.uint64(j % 64)
    return out


def _worker(rank, world, port, n, result):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc, k, s, m = _corpus(n)
    lo, hi = shard_range(n, rank, world)
    per = shard_range(n, 0, world)[1]
    words = (per + 63) // 64
    w = torch.from_numpy(_verdict_words(orc, k, s, m, lo, hi, words).view(np.int64))
    g = gather_verdicts(w, world)
    slowest = max_over_ranks(float(rank + 1))
    if rank == 0:
        result.put((g.numpy().view(np.uint64).copy(), slowest))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges_cover_and_align():
    for n in (0, 1, 63, 64, 65, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c
            assert all(lo % 64 == 0 for lo, hi in rs if hi > lo)


@pytest.mark.timeout(300)
def test_two_rank_gloo_verdict_gather():
    n, world = 300, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, slowest = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    orc, k, s, m = _corpus(n)
    full = _verdict_words(orc, k, s, m, 0, n, (n + 63) // 64)
    per = shard_range(n, 0, world)[1]
    # rank r's words start at r * per / 64 (shards are 64-aligned)
    got = np.zeros_like(full)
    wpr = (per + 63) // 64
    for r in range(world):
        lo, hi = shard_range(n, r, world)
        for j in range((hi - lo + 63) // 64):
            got[lo // 64 + j] = gathered[r * wpr + j]
    assert np.array_equal(got, full)
    assert slowest == 2.0
