#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X Corda verification engine.

Default workload (BASELINE.json configs[1], "C2"): one step = one pass of the
hot path (`Crypto.isValid(EDDSA_ED25519_SHA512, ...)` over a batch, kernel K1)
over 2^24 Ed25519 (key, sig, 32-byte txId) tuples resident in HBM, 1% of them
corrupted / non-canonical with SURVEY.md §8(d)'s fixed catalogue, plus the
RCCL all-gather of the per-GPU verdict bitmasks when N > 1.

Other workloads (`--workload`), same contract, used for profiling the other rows:
  c3  mixed secp256k1 / P-256 ECDSA, 2^24 per GPU, 1% corrupted (kernel K2)
  c4  SignedTransaction.verifySignatures over synthetic cash-issue transactions
      (5 leaves, 1-3 Ed25519 signers): leaf SHA-256 + Merkle id + signatures
      + per-tx reduce (K3/K4/K1/K5); 10^7 / 8 txs per GPU by default.

Contract: `python bench.py --gpus N --steps K --warmup W`; rank 0 prints ONE
JSON line. N > 1 runs one rank per GPU: under torch.distributed.run (WORLD_SIZE
set, and it must equal N), or -- when WORLD_SIZE is unset -- bench.py starts
the N ranks itself as a child `torch.distributed.run` before anything touches
the GPU, relays rank 0's line and exits non-zero if any rank fails. Every rank
binds its host threads to its GPU's NUMA node before HIP starts
(corda_amd/numa.py) and records the node in `config`.
Weak scaling: every rank verifies its own batch; value = all ranks'
verifications / max-over-ranks wall time of the K timed steps. C5 also has a
strong-scaling mode, `--global-log2 G` (a fixed 2^28 stream split
over the ranks; "scaling": "strong").
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "signature verifications/sec (whole node, 1/2/4/8 GPU) + % integer-ALU peak"
# algorithmic work per verification, in limb-MACs
# (32x32->64 multiply-accumulates of schoolbook radix-2^32: 64 per field mul).
LIMB_MACS = {"ed25519": 198_000, "p256": 211_000, "secp256k1": 192_000}
# Integer-ALU peak: 256 CUs x 64 v_mad_u64_u32 lane-ops per CU-cycle x 2.4 GHz
# (per-CU rate measured: profiles/r01_int_rates.jsonl, 59-62 lane-ops/CU-cycle).
INT_MAC_PEAK_T = 256 * 64 * 2.4e9 / 1e12
# the MEASURED v_mad_u64_u32 throughput, 59.43 lane-ops per
# CU-cycle (profiles/r01_int_rates.jsonl, 8 independent chains, 2048 blocks),
# taken at the shader clock this run holds (clock_ghz; 2.4 GHz without a reading)
MAD_U64_LANE_OPS_PER_CU_CYCLE = 59.43
C4_LEAF_LENS = (450, 150, 140, 43, 55)  # SURVEY §8(d) C4 synthetic cash-issue component lengths


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import load_oracle  # oracle loader lives with the tests (checker only)
    return load_oracle()


def _cgroup_cpus():
    """CPUs granted by the cgroup's CPU quota (cgroup v2 cpu.max, v1 cfs files), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else max(1, -(-q // per))
    except (OSError, ValueError):
        return None


_NUMA = {}  # this rank's NUMA binding (corda_amd.numa.bind_rank), set in main()


def _cores():
    """Host threads for the CPU legs: every CPU this process may run on
    (sched_getaffinity), capped by the cgroup CPU quota when one is set (more
    threads than the quota only time-slice), shared evenly by the ranks that
    share those CPUs (the ranks bound to the same NUMA node, else all local ranks)."""
    n = len(os.sched_getaffinity(0))
    q = _cgroup_cpus()
    if q:
        n = min(n, q)
    share = _NUMA.get("ranks_on_node") or int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    return max(1, n // share)


def _cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": _cgroup_cpus(),
            "os_cpu_count": os.cpu_count()}


def _ed_oracle_check(eng_status, keys, sigs, msgs, idx):
    """Oracle statuses for the lanes idx of a device Ed25519 batch vs the GPU's
    (oracle/c, the checker: construction-open lanes, e.g. slide()-dependent S)."""
    import numpy as np
    orc = _oracle()
    m = int(idx.numel())
    if m == 0:
        return {"lanes": 0, "mismatches": 0}
    k = keys[idx].cpu().numpy().copy()
    s = sigs[idx].cpu().numpy().copy()
    g = msgs[idx].cpu().numpy().copy()
    out = np.zeros(m, np.uint8)
    orc.oracle_ed25519_verify_batch(m, k.ctypes.data, s.ctypes.data, g.ctypes.data, g.shape[1], out.ctypes.data,
                                    _cores())
    got = eng_status[idx].cpu().numpy()
    return {"lanes": m, "mismatches": int((out != got).sum()), "oracle_accepted": int((out == 0).sum())}


def _ec_oracle_check(status, scheme, keys, key_len, sigs, sig_len, msgs, idx):
    """Oracle statuses for lanes idx of a slot-layout ECDSA batch vs the GPU's."""
    import numpy as np
    orc = _oracle()
    m = int(idx.numel())
    if m == 0:
        return {"lanes": 0, "mismatches": 0}
    sc = scheme[idx].cpu().numpy().copy()
    kl = key_len[idx].cpu().numpy().astype(np.uint64)
    sl = sig_len[idx].cpu().numpy().astype(np.uint64)
    K = keys[idx].cpu().numpy()
    S = sigs[idx].cpu().numpy()
    M = np.ascontiguousarray(msgs[idx].cpu().numpy())
    kb = np.ascontiguousarray(np.concatenate([K[i, :kl[i]] for i in range(m)]))
    sb = np.ascontiguousarray(np.concatenate([S[i, :sl[i]] for i in range(m)]))
    ko = np.zeros(m + 1, np.uint64)
    so = np.zeros(m + 1, np.uint64)
    ko[1:] = np.cumsum(kl)
    so[1:] = np.cumsum(sl)
    mo = np.arange(m + 1, dtype=np.uint64) * M.shape[1]
    out = np.zeros(m, np.uint8)
    orc.oracle_ecdsa_verify_batch(m, sc.ctypes.data, kb.ctypes.data, ko.ctypes.data, sb.ctypes.data, so.ctypes.data,
                                  M.ctypes.data, mo.ctypes.data, out.ctypes.data, _cores())
    got = status[idx].cpu().numpy()
    return {"lanes": m, "mismatches": int((out != got).sum()), "oracle_accepted": int((out == 0).sum())}


# ---- C2: Ed25519 ---------------------------------------------------------------
class C2:
    # one step = the split verification pass: prep (decode A/R, SHA-512, lattice
    # reduction -> per-lane workspace) + ladder, one launch pair for the whole
    # 2^24-lane batch (the workspace holds 2^24 lanes, cordahip.cpp kEdWsLanes)
    kernel = "ed25519_prep_half_kernel + ed25519_ladder_half_kernel"
    pmc = "r06_pmc_c2.json"  # tools/gpu_pmc_step.sh -> tools/pmc_step.py: one timed step of this workload

    def __init__(self, eng, device, stream, rank, args):
        import torch
        from corda_amd.corpus import make_c2_corpus
        self.torch, self.eng, self.device, self.stream = torch, eng, device, stream
        self.n = n = 1 << args.batch_log2
        self.pubs, self.sigs, self.msgs, self.expected, _ = make_c2_corpus(eng, n, 0xC0DA0002 + rank, device,
                                                                           stream=stream)
        self.status = torch.empty(n, dtype=torch.uint8, device=device)
        self.verdict = torch.empty((n + 63) // 64, dtype=torch.int64, device=device)
        self.units = n
        self.macs = LIMB_MACS["ed25519"]
        self.workload = ("C2: Ed25519 batch of 2^%d sigs per GPU, 32-byte txIds, 1%% corrupted/non-canonical"
                         % args.batch_log2)
        self.data = ("synthetic: seeded RFC 8032 tuples signed on the GPU (cordahip_ed25519_sign_device), "
                     "1% corrupted per SURVEY §8(d) C2")
        self.config = {"batch_per_gpu": n, "msg_len": 32, "corrupt_frac": 0.01}

    def step(self):
        self.eng.ed25519_verify_device(self.pubs, self.sigs, self.msgs, self.status, self.verdict, device=0,
                                       stream=self.stream)

    def check(self):
        # every lane is checked: lanes whose status the corpus construction fixes
        # against it, the construction-open ones (S + kL, slide()-dependent) against
        # the C oracle, so the whole 2^24-lane status vector is bit-exact attested
        known = self.expected >= 0
        open_ = (self.expected < 0).nonzero().flatten()
        orc = _ed_oracle_check(self.status, self.pubs, self.sigs, self.msgs, open_)
        return {"mismatches_vs_construction": int((self.status[known].to(self.torch.int16)
                                                   != self.expected[known]).sum()),
                "construction_lanes": int(known.sum()),
                "mismatches_vs_oracle_open_lanes": orc["mismatches"], "open_lanes_oracle_checked": orc["lanes"],
                "lanes_checked": int(known.sum()) + orc["lanes"], "lanes": self.n,
                "accepted": int((self.status == 0).sum()), "corrupted": int((self.expected != 0).sum())}

    def cpu_baseline(self, sample):
        import numpy as np
        orc = _oracle()
        k = self.pubs[:sample].cpu().numpy().copy()
        s = self.sigs[:sample].cpu().numpy().copy()
        m = self.msgs[:sample].cpu().numpy().copy()
        out = np.zeros(sample, np.uint8)
        cores = _cores()
        t0 = time.perf_counter()
        orc.oracle_ed25519_verify_batch(sample, k.ctypes.data, s.ctypes.data, m.ctypes.data, 32, out.ctypes.data,
                                        cores)
        dt = time.perf_counter() - t0
        one = min(sample, 4096)
        out1 = np.zeros(one, np.uint8)
        t1 = time.perf_counter()
        orc.oracle_ed25519_verify_batch(one, k.ctypes.data, s.ctypes.data, m.ctypes.data, 32, out1.ctypes.data, 1)
        dt1 = time.perf_counter() - t1
        mism = int((out != self.status[:sample].cpu().numpy()).sum())
        return {"value": sample / dt, "unit": "verifications/s", "cores": cores, "kind": "port",
                "sample": "first %d tuples of the rank-0 C2 batch (same corpus, 1%% corrupted), %d threads; "
                          "single-thread rate on %d tuples: %.0f/s" % (sample, cores, one, one / dt1),
                "single_thread_value": one / dt1, "wall_s": dt, "gpu_vs_port_mismatches_on_sample": mism}


# ---- C1: the CPU reference path's own workload, all valid ------------------------
class C1(C2):
    """2^20 tuples, seed_i = SHA-256("C1" || u64 i), msg_i =
    SHA-256("C1msg" || u64 i), key/sig by RFC 8032 (signed on the GPU). The GPU
    line verifies the same 2^20 tuples; cpu_baseline times the C restatement at 1
    thread and at `cores` threads, and OpenSSL 3 EVP_DigestVerify (an independent
    CPU Ed25519, raw-key decode included per call like Crypto.doVerify's key
    handling) on a sample, all on the same tuples."""
    pmc = "r06_pmc_c1.json"  # tools/gpu_pmc_step.sh -> tools/pmc_step.py: one timed step of this workload

    def __init__(self, eng, device, stream, rank, args):
        import hashlib
        import numpy as np
        import torch
        self.torch, self.eng, self.device, self.stream = torch, eng, device, stream
        self.n = n = 1 << args.batch_log2
        base = rank * n
        seeds = np.frombuffer(b"".join(hashlib.sha256(b"C1" + (base + i).to_bytes(8, "little")).digest()
                                       for i in range(n)), np.uint8).reshape(n, 32)
        msgs = np.frombuffer(b"".join(hashlib.sha256(b"C1msg" + (base + i).to_bytes(8, "little")).digest()
                                      for i in range(n)), np.uint8).reshape(n, 32)
        sd = torch.from_numpy(seeds.copy()).to(device)
        self.msgs = torch.from_numpy(msgs.copy()).to(device)
        self.pubs = torch.empty((n, 32), dtype=torch.uint8, device=device)
        self.sigs = torch.empty((n, 64), dtype=torch.uint8, device=device)
        eng.ed25519_sign_device(sd, self.msgs, self.pubs, self.sigs, device=0, stream=stream)
        torch.cuda.synchronize(device)
        self.expected = torch.zeros(n, dtype=torch.int16, device=device)
        self.status = torch.empty(n, dtype=torch.uint8, device=device)
        self.verdict = torch.empty((n + 63) // 64, dtype=torch.int64, device=device)
        self.units = n
        self.macs = LIMB_MACS["ed25519"]
        self.workload = "C1: Crypto.doVerify EDDSA_ED25519_SHA512 over 2^%d valid (key, sig, 32-byte txId) tuples" \
                        % args.batch_log2
        self.data = "synthetic: SURVEY §8(d) C1 seeds/messages, RFC 8032 keys and signatures made on the GPU"
        self.config = {"batch_per_gpu": n, "msg_len": 32, "corrupt_frac": 0.0}

    def cpu_baseline(self, sample):
        out = C2.cpu_baseline(self, sample)
        out["sample"] = out["sample"].replace("C2 batch (same corpus, 1% corrupted)", "C1 set (all valid)")
        # OpenSSL 3 (libcrypto.so.3, present on the box) as an independent CPU reference:
        # oracle/c/libosslbatch.so, pthreads over EVP_PKEY_new_raw_public_key + EVP_DigestVerify
        try:
            import ctypes
            import numpy as np
            so = os.path.join(ROOT, "oracle", "c", "libosslbatch.so")
            if not os.path.exists(so):
                subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle", "c"), "libosslbatch.so"])
            ossl = ctypes.CDLL(so)
            ossl.openssl_ed25519_verify_batch.argtypes = [ctypes.c_size_t] + [ctypes.c_void_p] * 3 + [
                ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
            k = self.pubs[:sample].cpu().numpy().copy()
            s = self.sigs[:sample].cpu().numpy().copy()
            m = self.msgs[:sample].cpu().numpy().copy()
            ok = np.zeros(sample, np.uint8)
            cores = _cores()
            t0 = time.perf_counter()
            rc = ossl.openssl_ed25519_verify_batch(sample, k.ctypes.data, s.ctypes.data, m.ctypes.data, 32,
                                                   ok.ctypes.data, cores)
            dt = time.perf_counter() - t0
            one = min(sample, 8192)
            t1 = time.perf_counter()
            ossl.openssl_ed25519_verify_batch(one, k.ctypes.data, s.ctypes.data, m.ctypes.data, 32,
                                              ok.ctypes.data, 1)
            dt1 = time.perf_counter() - t1
            out["openssl"] = {"value": sample / dt, "cores": cores, "sample": sample, "accepted": int(ok.sum()),
                              "single_thread_value": one / dt1, "rc": rc,
                              "note": "OpenSSL 3 EVP_PKEY_new_raw_public_key + EVP_DigestVerify per tuple, C pthreads "
                                      "(oracle/c/openssl_batch.c); an independent RFC 8032 implementation"}
        except Exception as e:  # noqa: BLE001 - the independent reference is optional on a box without libcrypto
            out["openssl"] = {"error": "%s: %s" % (type(e).__name__, e)}
        return out


# ---- C3: mixed secp256k1 / P-256 ECDSA ----------------------------------------
class C3:
    kernel = "ecdsa_prep_kernel + ecdsa_inv_kernel + ecdsa_ladder_kernel"
    pmc = "r06_pmc_c3.json"  # tools/gpu_pmc_step.sh -> tools/pmc_step.py: one timed step of this workload

    def __init__(self, eng, device, stream, rank, args):
        import torch
        from corda_amd.corpus import make_c3_corpus
        self.torch, self.eng, self.device, self.stream = torch, eng, device, stream
        self.n = n = 1 << args.batch_log2
        (self.scheme, self.keys, self.key_len, self.sigs, self.sig_len, self.msgs, self.expected,
         self.cats) = make_c3_corpus(eng, n, 0xC0DA0003 + rank, device, stream=stream)
        self.status = torch.empty(n, dtype=torch.uint8, device=device)
        self.verdict = torch.empty((n + 63) // 64, dtype=torch.int64, device=device)
        self.units = n
        self.macs = (LIMB_MACS["p256"] + LIMB_MACS["secp256k1"]) // 2
        self.workload = ("C3: mixed ECDSA_SECP256K1_SHA256 / ECDSA_SECP256R1_SHA256 (interleaved 50/50) batch of "
                         "2^%d sigs per GPU, 32-byte txIds, 1%% corrupted, ~10%% compressed keys, ~50%% high-S"
                         % args.batch_log2)
        self.data = ("synthetic: seeded keys/sigs made on the GPU (cordahip_ecdsa_sign_device), 1% corrupted per "
                     "SURVEY §8(d) C3 (DER malformations, r/s = 0, r/s >= n, bit flips, off-curve keys)")
        self.config = {"batch_per_gpu": n, "msg_len": 32, "corrupt_frac": 0.01}

    def step(self):
        self.eng.ecdsa_verify_device(self.scheme, self.keys, self.key_len, self.sigs, self.sig_len, self.msgs,
                                     self.status, self.verdict, device=0, stream=self.stream)

    def check(self):
        # exact-status lanes vs the construction; REJECT_ANY lanes (bit flips whose
        # status -- BAD_SIG or MALFORMED_SIG -- the flip decides) vs the C oracle
        st = self.status.to(self.torch.int16)
        exact = self.expected >= 0
        open_ = (self.expected < 0).nonzero().flatten()
        orc = _ec_oracle_check(self.status, self.scheme, self.keys, self.key_len, self.sigs, self.sig_len, self.msgs,
                               open_)
        return {"mismatches_vs_construction": int((st[exact] != self.expected[exact]).sum()),
                "construction_lanes": int(exact.sum()),
                "mismatches_vs_oracle_open_lanes": orc["mismatches"], "open_lanes_oracle_checked": orc["lanes"],
                "lanes_checked": int(exact.sum()) + orc["lanes"], "lanes": self.n,
                "accepted": int((self.status == 0).sum()), "corrupted": int((self.expected != 0).sum()),
                "compressed_valid": int(self.cats["compressed_valid"].numel())}

    def cpu_baseline(self, sample):
        import numpy as np
        orc = _oracle()
        sc = self.scheme[:sample].cpu().numpy().copy()
        kl = self.key_len[:sample].cpu().numpy().astype(np.uint64)
        sl = self.sig_len[:sample].cpu().numpy().astype(np.uint64)
        # CSR views over the fixed slots: offsets point at each slot, lengths from key_len / sig_len
        K = self.keys[:sample].cpu().numpy().copy()
        S = self.sigs[:sample].cpu().numpy().copy()
        M = self.msgs[:sample].cpu().numpy().copy()
        kb = np.ascontiguousarray(np.concatenate([K[i, :kl[i]] for i in range(sample)]))
        sb = np.ascontiguousarray(np.concatenate([S[i, :sl[i]] for i in range(sample)]))
        ko = np.zeros(sample + 1, np.uint64)
        so = np.zeros(sample + 1, np.uint64)
        ko[1:] = np.cumsum(kl)
        so[1:] = np.cumsum(sl)
        mo = (np.arange(sample + 1, dtype=np.uint64) * 32)
        out = np.zeros(sample, np.uint8)
        cores = _cores()
        t0 = time.perf_counter()
        orc.oracle_ecdsa_verify_batch(sample, sc.ctypes.data, kb.ctypes.data, ko.ctypes.data, sb.ctypes.data,
                                      so.ctypes.data, M.ctypes.data, mo.ctypes.data, out.ctypes.data, cores)
        dt = time.perf_counter() - t0
        mism = int((out != self.status[:sample].cpu().numpy()).sum())
        return {"value": sample / dt, "unit": "verifications/s", "cores": cores, "kind": "port",
                "sample": "first %d tuples of the rank-0 C3 batch (BouncyCastle-1.57 restatement in C, "
                          "%d threads)" % (sample, cores),
                "wall_s": dt, "gpu_vs_port_mismatches_on_sample": mism}


# ---- C4: SignedTransaction.verifySignatures on cash-issue transactions --------
class C4:
    kernel = "sha256_leaves + merkle_root + ed25519 prep/ladder + tx_reduce"
    pmc = "r06_pmc_c4.json"  # tools/gpu_pmc_step.sh -> tools/pmc_step.py: one timed step of this workload

    def __init__(self, eng, device, stream, rank, args):
        import torch
        self.torch, self.eng, self.device, self.stream = torch, eng, device, stream
        ntx = args.c4_txs
        g = torch.Generator(device=device)
        g.manual_seed(0xC0DA0004 + rank)
        nl = len(C4_LEAF_LENS)
        self.native = bool(getattr(args, "native_leaves", False)) or bool(getattr(args, "device_encode", False))
        self.device_encode = bool(getattr(args, "device_encode", False))
        nsig = torch.randint(1, 4, (ntx,), dtype=torch.int64, device=device, generator=g)
        self.tx_sig_off = torch.zeros(ntx + 1, dtype=torch.int64, device=device)
        self.tx_sig_off[1:] = torch.cumsum(nsig, 0)
        ns = int(self.tx_sig_off[-1])
        seeds = torch.randint(0, 256, (ns, 32), dtype=torch.uint8, device=device, generator=g)
        if self.native:
            # real-shaped leaves: the five cash-issue components written by
            # cordahip_kryo_encode; the issuer / command signer / mustSign key is the
            # transaction's first signer, whose public key comes from a signing pass
            from corda_amd.corpus import cash_issue_items, make_cash_issue_leaves
            first = self.tx_sig_off[:-1]
            pubs0 = torch.empty((ntx, 32), dtype=torch.uint8, device=device)
            scratch = torch.empty((ntx, 64), dtype=torch.uint8, device=device)
            eng.ed25519_sign_device(seeds[first].contiguous(), torch.zeros((ntx, 32), dtype=torch.uint8, device=device),
                                    pubs0, scratch, stream=stream)
            torch.cuda.synchronize(device)
            rng = np.random.default_rng(0xC0DA0004 + rank)
            comp = (pubs0.cpu().numpy(), rng.integers(0, 256, (ntx, 32), dtype=np.uint8),
                    rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(1, 10**9, ntx),
                    rng.integers(-2**63, 2**63 - 1, ntx))
            del pubs0, scratch
            if self.device_encode:
                # the components' payloads stay in HBM; every step hashes their leaves on the
                # GPU from the encoder's templates (cordahip_signed_txcomp_verify_ed25519_device:
                # items with payload offsets); the leaves themselves are written only by the
                # check (cordahip_kryo_encode_device: items with device pointers)
                blob, items, self.layout = cash_issue_items(*comp)
                self.host_blob, self.host_items = blob, items
                self.d_blob = torch.from_numpy(blob).to(device)
                it = items.reshape(-1).copy()
                self.d_items_off = torch.from_numpy(it.view(np.uint8).copy()).to(device)
                it["data"] += np.uint64(self.d_blob.data_ptr())
                self.d_items = torch.from_numpy(it.view(np.uint8)).to(device)
                self.n_items = it.size
                self.leaf_off = torch.zeros(self.n_items + 1, dtype=torch.int64, device=device)
                self.kstatus = torch.zeros(self.n_items, dtype=torch.uint8, device=device)
                eng.kryo_encode_device(self.d_items, self.n_items, None, self.leaf_off, self.kstatus, group=nl,
                                       stream=stream)  # sizes only
                torch.cuda.synchronize(device)
                self.leaf_bytes = torch.empty(int(self.leaf_off[-1]), dtype=torch.uint8, device=device)
            else:
                blob, off = make_cash_issue_leaves(*comp, threads=min(16, _cores()))
                self.leaf_bytes = torch.from_numpy(blob).to(device)
                self.leaf_off = torch.from_numpy(off.astype(np.int64)).to(device)
                del blob, off
        else:
            per_tx = sum(C4_LEAF_LENS)
            self.leaf_bytes = torch.randint(0, 256, (ntx * per_tx,), dtype=torch.uint8, device=device, generator=g)
            lens = torch.tensor(C4_LEAF_LENS, dtype=torch.int64, device=device).repeat(ntx)
            self.leaf_off = torch.zeros(ntx * nl + 1, dtype=torch.int64, device=device)
            self.leaf_off[1:] = torch.cumsum(lens, 0)
        self.tx_leaf_off = torch.arange(ntx + 1, dtype=torch.int64, device=device) * nl
        self.keys = torch.zeros((ns, 32), dtype=torch.uint8, device=device)
        self.sigs = torch.zeros((ns, 64), dtype=torch.uint8, device=device)
        self.txid = torch.empty((ntx, 32), dtype=torch.uint8, device=device)
        self.tx_status = torch.empty(ntx, dtype=torch.uint8, device=device)
        self.first_bad = torch.empty(ntx, dtype=torch.int64, device=device)
        self.sig_status = torch.empty(ns, dtype=torch.uint8, device=device)
        C4.step(self)  # computes the ids (signatures still blank)
        torch.cuda.synchronize(device)
        tx_of_sig = torch.repeat_interleave(torch.arange(ntx, device=device), nsig)
        msgs = self.txid[tx_of_sig].contiguous()
        eng.ed25519_sign_device(seeds, msgs, self.keys, self.sigs, stream=stream)
        torch.cuda.synchronize(device)
        del seeds, msgs
        # 0.5% of signatures: one bit of R flipped; 0.5% of transactions: one leaf byte flipped
        self.exp_status = torch.zeros(ntx, dtype=torch.uint8, device=device)
        self.exp_bad = torch.full((ntx,), -1, dtype=torch.int64, device=device)
        bad_sig = torch.randperm(ns, device=device, generator=g)[:max(1, ns // 200)]
        bit = torch.randint(0, 256, (bad_sig.numel(),), device=device, generator=g)
        self.sigs[bad_sig, bit // 8] ^= (1 << (bit % 8)).to(torch.uint8)
        t_bad = tx_of_sig[bad_sig]
        idx_in_tx = bad_sig - self.tx_sig_off[t_bad]
        self.exp_status[t_bad] = 1
        self.exp_bad.scatter_reduce_(0, t_bad, idx_in_tx, reduce="amin", include_self=False)
        bad_tx = torch.randperm(ntx, device=device, generator=g)[:max(1, ntx // 200)]
        if self.device_encode:  # a flipped owner-key byte in the component: the re-encoded leaf differs
            pos = (self.layout["owner_key"] + bad_tx * self.layout["cash_stride"]
                   + torch.randint(0, 32, (bad_tx.numel(),), device=device, generator=g))
            self.d_blob[pos] ^= 1
        else:
            pos = self.leaf_off[bad_tx * nl] + torch.randint(0, C4_LEAF_LENS[0], (bad_tx.numel(),), device=device,
                                                             generator=g)  # inside the output leaf (>= 450 B either way)
            self.leaf_bytes[pos] ^= 1
        self.exp_status[bad_tx] = 1
        self.exp_bad[bad_tx] = 0
        self.ntx, self.ns = ntx, ns
        self.units = ns
        self.macs = LIMB_MACS["ed25519"]
        leaves = ("native Kryo leaves (cordahip_kryo_encode%s: TransactionState<Cash.State>, issue Command, notary "
                  "Party, mustSign key, TransactionType; %.0f B per tx)"
                  % ("_device every step, from the components in HBM" if self.device_encode else "",
                     self.leaf_bytes.numel() / ntx)
                  if self.native else "5 leaves of %s B" % list(C4_LEAF_LENS))
        self.workload = ("C4: SignedTransaction.verifySignatures on %d synthetic cash-issue txs per GPU "
                         "(%s, 1-3 Ed25519 signers; leaf SHA-256 + Merkle id + sigs + per-tx reduce)" % (ntx, leaves))
        self.data = (("synthetic: seeded cash-issue components serialised natively (Kryo 4 restatement, parity "
                      "unpinned beyond the key bytes)" if self.native else
                      "synthetic: seeded random leaf bytes of the SURVEY §8(d) C4 lengths") +
                     ", signatures made on the GPU over the GPU-computed ids; 0.5% sigs and 0.5% txs corrupted")
        self.config = {"txs_per_gpu": ntx, "sigs_per_gpu": ns,
                       "leaf_bytes_per_tx": round(self.leaf_bytes.numel() / ntx, 1), "native_leaves": self.native,
                       "device_encode": self.device_encode}
        if self.device_encode:
            self.kernel = ("cordahip_signed_txcomp_verify_ed25519_device: kryo_shape + kryo_hash (leaf hashes from the "
                           "templates) + merkle_root + ed25519 prep/ladder + tx_reduce")
            self.pmc = "r06_pmc_c4de.json"  # its own step: the id chain from components included
            self.config["component_bytes_per_tx"] = round(self.d_blob.numel() / ntx, 1)
        if not self.native:
            self.config["leaf_lens"] = list(C4_LEAF_LENS)

    def step(self):
        if self.device_encode:
            self.eng.signed_txcomp_verify_ed25519_device(
                self.d_items_off, self.n_items, self.d_blob, self.tx_leaf_off, self.tx_sig_off, self.keys, self.sigs,
                self.txid, self.tx_status, self.first_bad, self.sig_status, group=len(C4_LEAF_LENS), device=0,
                stream=self.stream)
            return
        self.eng.signed_tx_verify_ed25519_device(self.leaf_bytes, self.leaf_off, self.tx_leaf_off, self.tx_sig_off,
                                                 self.keys, self.sigs, self.txid, self.tx_status, self.first_bad,
                                                 self.sig_status, device=0, stream=self.stream)

    def check(self):
        out = {"mismatches_vs_construction": int((self.tx_status != self.exp_status).sum())
               + int((self.first_bad != self.exp_bad).sum()),
               "accepted_txs": int((self.tx_status == 0).sum()), "txs": self.ntx, "sigs": self.ns}
        if getattr(self, "device_encode", False):
            # (1) every leaf written by the GPU encoder (cordahip_kryo_encode_device, untimed) and
            # the leaf-level device path over them: all ids, statuses and first_bad_sig equal the
            # component call's; (2) the leaves of the first 20,000 transactions against the host
            # encoder (cordahip_kryo_encode) over the same (corrupted) components
            from corda_amd import _lib
            t = self.torch
            self.eng.kryo_encode_device(self.d_items, self.n_items, self.leaf_bytes, self.leaf_off, self.kstatus,
                                        group=len(C4_LEAF_LENS), device=0, stream=self.stream)
            lp = [t.empty_like(x) for x in (self.txid, self.tx_status, self.first_bad, self.sig_status)]
            self.eng.signed_tx_verify_ed25519_device(self.leaf_bytes, self.leaf_off, self.tx_leaf_off, self.tx_sig_off,
                                                     self.keys, self.sigs, *lp, device=0, stream=self.stream)
            t.cuda.synchronize(self.device)
            out["mismatches_vs_leaf_path"] = (int((lp[0] != self.txid).any(dim=1).sum()) + int((lp[1] != self.tx_status).sum())
                                              + int((lp[2] != self.first_bad).sum()) + int((lp[3] != self.sig_status).sum()))
            k = min(self.ntx, 20000) * len(C4_LEAF_LENS)
            blob = self.d_blob.cpu().numpy()
            it = self.host_items.reshape(-1)[:k].copy()
            it["data"] += np.uint64(blob.ctypes.data)
            hb, ho = _lib.kryo_encode_array(it)
            lo = self.leaf_off[:k + 1].cpu().numpy().astype(np.uint64)
            out["kryo_item_errors"] = int((self.kstatus != 0).sum())
            out["leaf_mismatches_vs_host_encoder"] = int(not (np.array_equal(lo, ho) and np.array_equal(
                self.leaf_bytes[:int(lo[-1])].cpu().numpy(), hb)))
            out["leaves_checked_vs_host_encoder"] = k
        return out

    def cpu_baseline(self, sample):
        import ctypes
        import numpy as np
        orc = _oracle()
        ntx = max(1, min(self.ntx, sample // 2))
        lb = self.leaf_bytes[:int(self.leaf_off[ntx * len(C4_LEAF_LENS)])].cpu().numpy().copy()
        lo = self.leaf_off[:ntx * len(C4_LEAF_LENS) + 1].cpu().numpy().astype(np.uint64)
        so = self.tx_sig_off[:ntx + 1].cpu().numpy()
        ns = int(so[-1])
        K = self.keys[:ns].cpu().numpy().copy()
        S = self.sigs[:ns].cpu().numpy().copy()
        ids = np.zeros((ntx, 32), np.uint8)
        out = np.zeros(ns, np.uint8)
        cores = _cores()
        nl = len(C4_LEAF_LENS)
        t0 = time.perf_counter()
        for t in range(ntx):
            orc.oracle_tx_id(lb.ctypes.data, lo[t * nl:].ctypes.data, nl, ctypes.cast(ids[t].ctypes.data, ctypes.c_char_p))
        M = ids[np.repeat(np.arange(ntx), np.diff(so))]
        orc.oracle_ed25519_verify_batch(ns, K.ctypes.data, S.ctypes.data, M.ctypes.data, 32, out.ctypes.data, cores)
        dt = time.perf_counter() - t0
        mism = int((out != self.sig_status[:ns].cpu().numpy()).sum())
        return {"value": ns / dt, "unit": "verifications/s", "cores": cores, "kind": "port",
                "sample": "first %d txs (%d sigs) of the rank-0 C4 batch: tx ids single-threaded, signatures on %d "
                          "threads" % (ntx, ns, cores),
                "wall_s": dt, "txs_per_s": ntx / dt, "gpu_vs_port_mismatches_on_sample": mism}


# ---- C5: verifier-module queue drain, mixed schemes, pinned host memory -------
class C5:
    kernel = "ed25519 prep/ladder + ecdsa prep/inv/ladder, 3-stage H2D/kernel/D2H pipeline"
    pmc = "r06_pmc_c5.json"  # tools/gpu_pmc_step.sh -> tools/pmc_step.py: one timed step of this workload
    host_timed = True  # the drain is synchronous and owns its streams: wall time, PCIe included

    def __init__(self, eng, device, stream, rank, args):
        import torch
        from corda_amd.corpus import make_c2_corpus, make_c3_corpus
        self.torch, self.eng, self.device = torch, eng, device
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.verdict = None  # built per step when N > 1 (the all-gather operand)
        n = 1 << args.batch_log2
        n_ec = n // 5  # 80% Ed25519 / 10% P-256 / 10% secp256k1
        n_ed = n - n_ec
        pubs, sigs, msgs, self.exp_ed, _ = make_c2_corpus(eng, n_ed, 0xC0DA0005 + rank, device, stream=stream)
        (scheme, keys, key_len, esigs, sig_len, emsgs, self.exp_ec,
         _) = make_c3_corpus(eng, n_ec, 0xC0DA0105 + rank, device, stream=stream)
        torch.cuda.synchronize(device)
        pin = lambda t: t.cpu().contiguous().pin_memory()
        self.ed = [pin(t) for t in (pubs, sigs, msgs)] + [torch.zeros(n_ed, dtype=torch.uint8).pin_memory()]
        self.ec = [pin(t) for t in (scheme, keys, key_len, esigs, sig_len, emsgs)] + \
                  [torch.zeros(n_ec, dtype=torch.uint8).pin_memory()]
        self.exp_ed, self.exp_ec = self.exp_ed.cpu(), self.exp_ec.cpu()
        del pubs, sigs, msgs, scheme, keys, key_len, esigs, sig_len, emsgs
        self.n_ed, self.n_ec = n_ed, n_ec
        # strong scaling (--global-log2 G): the rank's share of a fixed 2^G batch
        # is its 2^batch_log2 corpus streamed `passes` times per step
        self.passes = 1
        if args.global_log2:
            world = int(os.environ.get("WORLD_SIZE", "1"))
            share = (1 << args.global_log2) // world
            if share % n:
                raise SystemExit("--global-log2: 2^%d / %d ranks is not a multiple of 2^%d"
                                 % (args.global_log2, world, args.batch_log2))
            self.passes = share // n
        self.units = n * self.passes
        self.macs = (n_ed * LIMB_MACS["ed25519"] + n_ec * (LIMB_MACS["p256"] + LIMB_MACS["secp256k1"]) // 2) // n
        self.workload = ("C5: verifier-module queue drain, 2^%d mixed sigs per GPU per step (80%% Ed25519, 10%% P-256, "
                         "10%% secp256k1, 1%% corrupted) streamed from pinned host memory, H2D/D2H included"
                         % args.batch_log2)
        self.data = "synthetic: C2 and C3 corpora (GPU-signed), copied to pinned host memory before timing"
        self.config = {"batch_per_gpu": n * self.passes, "ed25519": n_ed, "ecdsa": n_ec, "chunk": int(os.environ.get("CORDAHIP_STREAM_CHUNK", 1 << 23)),
                       "stages": 3}
        if args.global_log2:
            self.workload += "; strong scaling: a fixed 2^%d global batch, this rank's share = %d passes" % (
                args.global_log2, self.passes)
            self.config["global_batch"] = 1 << args.global_log2

    def step(self):
        for _ in range(self.passes):
            self.eng.stream_verify(self.ed, self.ec)
        if self.world > 1:
            self.verdict = self._verdict_words()

    def _verdict_words(self):
        """The rank's verdict mask (bit i = lane i OK, Ed25519 lanes then ECDSA lanes)
        as device words, the operand of the step's RCCL all-gather: the
        drain leaves its statuses in pinned host memory, so they go H2D once and are
        packed on the GPU (~1 ms of a ~170 ms step)."""
        t = self.torch
        st = t.cat([self.ed[3], self.ec[6]]).to(self.device, non_blocking=True)
        return _pack_verdict(st)

    def check(self):
        t = self.torch
        st_ed = self.ed[3].to(t.int16)
        st_ec = self.ec[6].to(t.int16)
        k = self.exp_ed >= 0
        ex = self.exp_ec >= 0
        o_ed = _ed_oracle_check(self.ed[3], self.ed[0], self.ed[1], self.ed[2], (self.exp_ed < 0).nonzero().flatten())
        o_ec = _ec_oracle_check(self.ec[6], *self.ec[:6], (self.exp_ec < 0).nonzero().flatten())
        return {"mismatches_vs_construction": int((st_ed[k] != self.exp_ed[k]).sum())
                + int((st_ec[ex] != self.exp_ec[ex]).sum()),
                "construction_lanes": int(k.sum()) + int(ex.sum()),
                "mismatches_vs_oracle_open_lanes": o_ed["mismatches"] + o_ec["mismatches"],
                "open_lanes_oracle_checked": o_ed["lanes"] + o_ec["lanes"],
                "lanes_checked": int(k.sum()) + int(ex.sum()) + o_ed["lanes"] + o_ec["lanes"],
                "lanes": self.n_ed + self.n_ec,
                "accepted": int((st_ed == 0).sum()) + int((st_ec == 0).sum())}

    def cpu_baseline(self, sample):
        import numpy as np
        orc = _oracle()
        se, sc = sample - sample // 5, sample // 5
        k, s, m = (x[:se].numpy() for x in self.ed[:3])
        out = np.zeros(se, np.uint8)
        cores = _cores()
        t0 = time.perf_counter()
        orc.oracle_ed25519_verify_batch(se, k.ctypes.data, s.ctypes.data, m.ctypes.data, 32, out.ctypes.data, cores)
        t_ed = time.perf_counter() - t0
        sch, K, KL, S, SL, M = (x[:sc].numpy() for x in self.ec[:6])
        kb = np.ascontiguousarray(np.concatenate([K[i, :KL[i]] for i in range(sc)]))
        sb = np.ascontiguousarray(np.concatenate([S[i, :SL[i]] for i in range(sc)]))
        ko = np.zeros(sc + 1, np.uint64)
        so = np.zeros(sc + 1, np.uint64)
        ko[1:] = np.cumsum(KL.astype(np.uint64))
        so[1:] = np.cumsum(SL.astype(np.uint64))
        mo = np.arange(sc + 1, dtype=np.uint64) * 32
        out2 = np.zeros(sc, np.uint8)
        Mc = np.ascontiguousarray(M)
        t0 = time.perf_counter()
        orc.oracle_ecdsa_verify_batch(sc, sch.ctypes.data, kb.ctypes.data, ko.ctypes.data, sb.ctypes.data,
                                      so.ctypes.data, Mc.ctypes.data, mo.ctypes.data, out2.ctypes.data, cores)
        t_ec = time.perf_counter() - t0
        mism = int((out != self.ed[3][:se].numpy()).sum()) + int((out2 != self.ec[6][:sc].numpy()).sum())
        return {"value": sample / (t_ed + t_ec), "unit": "verifications/s", "cores": cores, "kind": "port",
                "sample": "first %d Ed25519 + %d ECDSA lanes of the rank-0 C5 queue (oracle/c, %d threads)"
                          % (se, sc, cores),
                "wall_s": t_ed + t_ec, "gpu_vs_port_mismatches_on_sample": mism}


# ---- the JVM's boundary: generic CSR batches in host memory ------------------
def _pinned(a):
    """numpy array -> page-locked CPU tensor (the JVM's direct ByteBuffers from
    cordahip_alloc_pinned are the same hipHostMalloc memory)."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory()


def _csr_rows(rows, lens):
    """[n, W] slots + per-lane lengths -> (blob, off[n+1]) with the bytes in lane order."""
    lens = lens.astype(np.int64)
    mask = np.arange(rows.shape[1])[None, :] < lens[:, None]
    off = np.zeros(rows.shape[0] + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    return rows[mask], off


class _HostSigBatch:
    """A cordahip_sig_batch over pinned host CSR arrays (scheme, key/sig/msg blobs + offsets).
    inflight K > 1: up to K cordahip_sig_submit tickets outstanding (a JVM's verifier
    workers or fibers submitting consecutive batches), each slot with its own status and
    verdict arrays; run() submits one and completes the oldest once K are out."""

    def __init__(self, scheme, kb, ko, sb, so, mb, mo, inflight=1):
        from corda_amd import _lib
        n = len(scheme)
        self.t = [_pinned(x) for x in (scheme, kb, ko, sb, so, mb, mo)]
        p = [x.data_ptr() for x in self.t]
        self.inflight = max(1, inflight)
        self.outs, self.bs = [], []
        for _ in range(self.inflight):
            st, vd = _pinned(np.zeros(n, np.uint8)), _pinned(np.zeros((n + 63) // 64, np.uint64))
            self.outs.append((st, vd))
            self.bs.append(_lib.SigBatch(n, *p, st.data_ptr(), vd.data_ptr(), 0,
                                         self.t[1].numel(), self.t[3].numel(), self.t[5].numel()))
        self.status, self.verdict = self.outs[0]
        self.b = self.bs[0]
        self.pending = []  # (ticket, slot), oldest first

    def run(self, eng):
        import ctypes
        from corda_amd._lib import check, lib
        if self.inflight == 1:
            check(lib().cordahip_sig_verify(eng.ctx, ctypes.byref(self.b)), "cordahip_sig_verify")
            return
        if len(self.pending) >= self.inflight:
            self._complete(eng)
        busy = {k for _, k in self.pending}
        slot = next(k for k in range(self.inflight) if k not in busy)
        t = ctypes.c_uint64()
        check(lib().cordahip_sig_submit(eng.ctx, ctypes.byref(self.bs[slot]), ctypes.byref(t)), "cordahip_sig_submit")
        self.pending.append((t.value, slot))

    def _complete(self, eng):
        from corda_amd._lib import check, lib
        t, slot = self.pending.pop(0)
        check(lib().cordahip_wait(eng.ctx, t, -1), "cordahip_wait")
        self.status, self.verdict = self.outs[slot]  # the last completed call's outputs

    def drain(self, eng):
        while self.pending:
            self._complete(eng)


class C2H(C2):
    """C2's corpus through the boundary the JVM calls: `Crypto.isValid` batches
    (Crypto.kt:534-541, doVerify semantics) as ONE cordahip_sig_verify over a
    2^24-lane CSR batch in pinned host memory. Timed region =
    the whole call: lane classification, host packing into pinned staging, PCIe
    both ways, the kernels, status scatter and verdict words."""
    kernel = "cordahip_sig_verify (host CSR batch): pack + H2D + ed25519 prep/ladder + D2H, pipelined"
    pmc = "r06_pmc_c2h.json"  # tools/gpu_pmc_step.sh -> tools/pmc_step.py: one timed step of this workload
    host_timed = True

    def __init__(self, eng, device, stream, rank, args):
        super().__init__(eng, device, stream, rank, args)
        n = self.n
        k, s, m = (x.cpu().numpy() for x in (self.pubs, self.sigs, self.msgs))
        ar = np.arange(n + 1, dtype=np.uint64)
        self.hb = _HostSigBatch(np.full(n, 4, np.uint8), k.reshape(-1), ar * 32, s.reshape(-1), ar * 64,
                                m.reshape(-1), ar * 32, inflight=getattr(args, "inflight", 1) or 1)
        self.workload = ("C2 via the JVM boundary: cordahip_sig_verify over a 2^%d-lane Ed25519 CSR batch in pinned "
                         "host memory (PCIe and host packing included), 1%% corrupted" % args.batch_log2)
        self.config = dict(self.config, boundary="cordahip_sig_verify", host_memory="pinned CSR",
                           inflight=self.hb.inflight)
        if self.hb.inflight > 1:
            self.workload += ("; up to %d cordahip_sig_submit calls outstanding (the timed region ends when every "
                              "call it submitted has completed)" % self.hb.inflight)

    def step(self):
        self.hb.run(self.eng)

    def drain(self):
        self.hb.drain(self.eng)

    def check(self):
        import torch
        st = self.hb.status
        self.status = st
        exp = self.expected.cpu()
        known = exp >= 0
        open_ = (exp < 0).nonzero().flatten()
        orc = _ed_oracle_check(st, self.pubs.cpu(), self.sigs.cpu(), self.msgs.cpu(), open_)
        ok = (st == 0)
        words = np.zeros((self.n + 63) // 64, np.uint64)
        bits = ok.numpy().reshape(-1, 64).astype(np.uint64) << np.arange(64, dtype=np.uint64)
        words[:] = bits.sum(axis=1, dtype=np.uint64)
        return {"mismatches_vs_construction": int((st[known].to(torch.int16) != exp[known]).sum()),
                "construction_lanes": int(known.sum()),
                "mismatches_vs_oracle_open_lanes": orc["mismatches"], "open_lanes_oracle_checked": orc["lanes"],
                "lanes_checked": int(known.sum()) + orc["lanes"], "lanes": self.n,
                "verdict_word_mismatches": int((words != self.hb.verdict.numpy()).sum()),
                "accepted": int(ok.sum()), "corrupted": int((exp != 0).sum())}

    def cpu_baseline(self, sample):
        self.status = self.hb.status
        return C2.cpu_baseline(self, sample)


class C3H(C3):
    """C3's corpus (mixed secp256k1 / P-256, DER signatures of 8-73 bytes, 33- or
    65-byte keys) through cordahip_sig_verify as a pinned host CSR batch."""
    kernel = "cordahip_sig_verify (host CSR batch): pack + H2D + ecdsa partition/prep/inv/ladders + D2H, pipelined"
    pmc = "r06_pmc_c3h.json"  # tools/gpu_pmc_step.sh -> tools/pmc_step.py: one timed step of this workload
    host_timed = True

    def __init__(self, eng, device, stream, rank, args):
        super().__init__(eng, device, stream, rank, args)
        n = self.n
        kb, ko = _csr_rows(self.keys.cpu().numpy(), self.key_len.cpu().numpy())
        sb, so = _csr_rows(self.sigs.cpu().numpy(), self.sig_len.cpu().numpy())
        ar = np.arange(n + 1, dtype=np.uint64)
        self.hb = _HostSigBatch(self.scheme.cpu().numpy(), kb, ko, sb, so, self.msgs.cpu().numpy().reshape(-1), ar * 32,
                                inflight=getattr(args, "inflight", 1) or 1)
        self.workload = ("C3 via the JVM boundary: cordahip_sig_verify over a 2^%d-lane mixed secp256k1 / P-256 CSR "
                         "batch in pinned host memory (PCIe and host packing included), 1%% corrupted" % args.batch_log2)
        self.config = dict(self.config, boundary="cordahip_sig_verify", host_memory="pinned CSR",
                           inflight=self.hb.inflight)
        if self.hb.inflight > 1:
            self.workload += ("; up to %d cordahip_sig_submit calls outstanding (the timed region ends when every "
                              "call it submitted has completed)" % self.hb.inflight)

    def step(self):
        self.hb.run(self.eng)

    def drain(self):
        self.hb.drain(self.eng)

    def check(self):
        self.status = self.hb.status
        dev = (self.scheme, self.keys, self.key_len, self.sigs, self.sig_len, self.msgs, self.expected)
        self.scheme, self.keys, self.key_len, self.sigs, self.sig_len, self.msgs, self.expected = (x.cpu() for x in dev)
        try:
            return C3.check(self)
        finally:
            self.scheme, self.keys, self.key_len, self.sigs, self.sig_len, self.msgs, self.expected = dev

    def cpu_baseline(self, sample):
        self.status = self.hb.status
        return C3.cpu_baseline(self, sample)


class C4H(C4):
    """C4's transactions through the boundary SignedTransaction.checkSignaturesAreValid
    maps to (SignedTransaction.kt:95-100): cordahip_tx_submit +
    cordahip_wait over pinned host CSR arrays (leaf bytes, per-tx leaves and
    signatures, CSR keys/sigs with scheme bytes). Timed: tx ids (leaf SHA-256 +
    Merkle) then every signature over its tx's id, PCIe both ways included."""
    kernel = "cordahip_tx_submit (host CSR): tx ids (sha256_leaves + merkle_root) then cordahip_sig_verify lanes"
    pmc = "r06_pmc_c4h.json"  # tools/gpu_pmc_step.sh -> tools/pmc_step.py: one timed step of this workload
    host_timed = True

    def __init__(self, eng, device, stream, rank, args):
        import argparse

        from corda_amd import _lib
        if getattr(args, "device_encode", False):
            raise SystemExit("--device-encode is a c4 option: c4h hands the library leaf bytes in host memory "
                             "(--components: the components, encoded on the GPU)")
        self.components = bool(getattr(args, "components", False))
        if self.components:  # the C4 corpus of cash-issue components (its device path encodes them each step)
            args = argparse.Namespace(**dict(vars(args), device_encode=True))
        super().__init__(eng, device, stream, rank, args)
        ntx, ns = self.ntx, self.ns
        ar = np.arange(ns + 1, dtype=np.uint64)
        sig_arrays = (np.full(ns, 4, np.uint8), self.keys.cpu().numpy().reshape(-1), ar * 32,
                      self.sigs.cpu().numpy().reshape(-1), ar * 64)
        # --inflight K: up to K calls outstanding (the JVM submitting consecutive
        # ResolveTransactionsFlow batches), each with its own output arrays; a step
        # submits one call, waiting first for the oldest when K are outstanding
        self.inflight = max(1, int(getattr(args, "inflight", 1) or 1))
        self.outs = [tuple(_pinned(x) for x in (np.zeros((ntx, 32), np.uint8), np.zeros(ntx, np.uint8),
                                                np.zeros(ns, np.uint8), np.zeros(ntx, np.int64)))
                     for _ in range(self.inflight)]
        self.h_txid, self.h_txst, self.h_sst, self.h_fb = self.outs[0]
        self.pending = []  # (ticket, slot), oldest first
        self.next_slot = 0
        self.bs = []
        if self.components:
            # what the JVM hands over instead of leaves: the Kryo items (data = offsets into the
            # payload) and the payload blob -- the corrupted owner keys included
            items = np.ascontiguousarray(self.host_items.reshape(-1))
            payload = self.d_blob.cpu().numpy()
            self.t = [_pinned(x) for x in (items.view(np.uint8), np.arange(0, 5 * ntx + 1, 5, dtype=np.uint64),
                                           payload, self.tx_sig_off.cpu().numpy().astype(np.uint64)) + sig_arrays]
            p = [x.data_ptr() for x in self.t]
            for txid, txst, sst, fb in self.outs:
                tb = _lib.TxcompBatch(ntx, p[0], p[1], p[2], payload.size, txid.data_ptr(), txst.data_ptr(), items.size)
                self.bs.append(_lib.SignedTxcompBatch(tb, p[3], p[4], p[5], p[6], p[7], p[8], sst.data_ptr(),
                                                      fb.data_ptr(), ns, self.t[5].numel(), self.t[7].numel()))
            self.pcie_tx_bytes = (items.nbytes + 8 * (5 * ntx + 1) + payload.size) / ntx
            what = ("the components of each tx (cordahip_txcomp_submit: %.0f B per tx of Kryo items and payload; "
                    "the GPU writes the %.0f B of leaves)" % (self.pcie_tx_bytes, self.leaf_bytes.numel() / ntx))
            self.kernel = ("cordahip_txcomp_submit (host CSR): per id slice kryo_shape + kryo_hash (the leaves' "
                           "SHA-256 from the encoder's templates; the full encoder + sha256_leaves when a shape is "
                           "new) + merkle_root, then the signature chunks")
            self.pmc = "r06_pmc_c4hc.json"  # tools/gpu_pmc_step.sh -> tools/pmc_step.py: one timed step of this workload
        else:
            self.t = [_pinned(x) for x in (
                self.leaf_bytes.cpu().numpy(), self.leaf_off.cpu().numpy().astype(np.uint64),
                self.tx_leaf_off.cpu().numpy().astype(np.uint64), self.tx_sig_off.cpu().numpy().astype(np.uint64))
                + sig_arrays]
            p = [x.data_ptr() for x in self.t]
            for txid, txst, sst, fb in self.outs:
                tb = _lib.TxidBatch(ntx, p[0], p[1], p[2], txid.data_ptr(), txst.data_ptr(), self.t[1].numel() - 1,
                                    self.t[0].numel())
                self.bs.append(_lib.SignedTxBatch(tb, p[3], p[4], p[5], p[6], p[7], p[8], sst.data_ptr(),
                                                  fb.data_ptr(), ns, self.t[5].numel(), self.t[7].numel()))
            self.pcie_tx_bytes = (self.leaf_bytes.numel() + 8 * (self.leaf_off.numel() + ntx + 1)) / ntx
            what = ("native Kryo leaves, %.0f B per tx" % (self.leaf_bytes.numel() / ntx) if self.native
                    else "5 leaves of %s B" % list(C4_LEAF_LENS))
        self.workload = ("C4 via the JVM boundary: %s over %d synthetic cash-issue txs per GPU in pinned "
                         "host CSR memory (%s, 1-3 Ed25519 signers; PCIe included)"
                         % ("cordahip_txcomp_submit" if self.components else "cordahip_tx_submit", ntx, what))
        self.config = dict(self.config, boundary=("cordahip_txcomp_submit" if self.components else "cordahip_tx_submit")
                           + " + cordahip_wait", host_memory="pinned CSR", components=self.components,
                           pcie_id_bytes_per_tx=round(self.pcie_tx_bytes, 1), inflight=self.inflight)
        if self.inflight > 1:
            self.workload += ("; up to %d calls outstanding (a step submits one; the timed region ends when every "
                              "call it submitted has completed)" % self.inflight)

    def _wait_oldest(self):
        import ctypes  # noqa: F401
        from corda_amd._lib import check, lib
        t, _ = self.pending.pop(0)
        check(lib().cordahip_wait(self.eng.ctx, t, -1), "cordahip_wait")

    def step(self):
        import ctypes
        from corda_amd._lib import check, lib
        if len(self.pending) >= self.inflight:
            self._wait_oldest()
        busy = {k for _, k in self.pending}
        slot = next(k for k in range(self.inflight) if k not in busy)
        t = ctypes.c_uint64()
        submit = lib().cordahip_txcomp_submit if self.components else lib().cordahip_tx_submit
        check(submit(self.eng.ctx, ctypes.byref(self.bs[slot]), ctypes.byref(t)), "cordahip_tx(comp)_submit")
        self.pending.append((t.value, slot))

    def drain(self):
        while self.pending:
            self._wait_oldest()

    def check(self):
        import torch  # noqa: F401
        self.drain()
        exp_st = self.exp_status.cpu()
        exp_bad = self.exp_bad.cpu()
        C4.step(self)  # the device-resident path over the same bytes: its ids
        self.torch.cuda.synchronize(self.device)
        txid = self.txid.cpu()
        # every output set (one per outstanding call) against the construction and the device path
        out = {"mismatches_vs_construction": sum(int((st != exp_st).sum()) + int((fb != exp_bad).sum())
                                                 for _, st, _, fb in self.outs),
               "txid_mismatches_vs_device_path": sum(int((ti != txid).any(dim=1).sum()) for ti, _, _, _ in self.outs),
               "output_sets_checked": len(self.outs),
               "accepted_txs": int((self.h_txst == 0).sum()), "txs": self.ntx, "sigs": self.ns}
        if self.components:  # the device path's leaves against the host encoder (C4 --device-encode's check)
            dev = C4.check(self)
            out["device_path_mismatches_vs_construction"] = dev["mismatches_vs_construction"]
            for k in ("kryo_item_errors", "leaf_mismatches_vs_host_encoder", "leaves_checked_vs_host_encoder"):
                out[k] = dev[k]
        return out

    def cpu_baseline(self, sample):
        self.sig_status = self.h_sst
        return C4.cpu_baseline(self, sample)


def _pack_verdict(status):
    """uint8 statuses (length a multiple of 64) -> int64 verdict words, bit i = (status[i] == 0)."""
    import torch
    ok = (status == 0).view(-1, 64).to(torch.int64)
    return (ok << torch.arange(64, device=status.device, dtype=torch.int64)).sum(dim=1)


class Stub:
    """CPU-only stand-in for the multi-process launcher tests (`--workload stub`,
    gloo, no GPU, no library): the same main() -- launcher, NUMA record, barrier
    + max-over-ranks timing, verdict all-gather -- around a trivial step (SHA-256
    of a 64 KiB buffer) over a seeded status vector."""
    kernel = "stub (CPU, no kernel)"
    pmc = None
    host_timed = True

    def __init__(self, eng, device, stream, rank, args):
        import hashlib
        import torch
        self.hashlib, self.torch = hashlib, torch
        if os.environ.get("CORDA_BENCH_STUB_FAIL_RANK") == str(rank):  # launcher test: a rank that dies
            raise SystemExit("stub: rank %d fails on request" % rank)
        self.n = n = 1 << min(args.batch_log2, 16)
        rng = np.random.default_rng(0xC0DA0000 + rank)
        self.status = torch.from_numpy((rng.random(n) < 0.01).astype(np.uint8))
        self.verdict = _pack_verdict(self.status)
        self.buf = rng.bytes(1 << 16)
        self.units = n
        self.macs = 0
        self.workload = "stub: launcher test, %d seeded lanes per rank, no GPU work" % n
        self.data = "synthetic: seeded statuses (numpy), CPU only"
        self.config = {"batch_per_gpu": n}

    def step(self):
        self.hashlib.sha256(self.buf).digest()

    def check(self):
        return {"mismatches_vs_construction": 0, "lanes": self.n, "accepted": int((self.status == 0).sum())}

    def cpu_baseline(self, sample):
        return {"value": None, "unit": "verifications/s", "cores": _cores(), "kind": "port",
                "sample": "stub workload: no CPU baseline"}


WORKLOADS = {"c1": C1, "c2": C2, "c3": C3, "c4": C4, "c5": C5, "c2h": C2H, "c3h": C3H, "c4h": C4H, "stub": Stub}


def _launch(n, argv):
    """Start N ranks as a child torch.distributed.run (this process has not touched
    the GPU, and never execs: the ranks are children), relay rank 0's JSON line,
    and return non-zero if any rank failed or the line is missing."""
    import signal
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + list(argv)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1, env=dict(os.environ, CORDA_BENCH_CHILD="1"))
    prev = signal.signal(signal.SIGTERM, lambda *_: p.send_signal(signal.SIGTERM))
    lines = []
    try:
        for line in p.stdout:
            if line.startswith("{") and '"metric"' in line:
                lines.append(line.strip())
            else:
                sys.stderr.write(line)
        rc = p.wait()
    except BaseException:
        p.terminate()
        p.wait()
        raise
    finally:
        signal.signal(signal.SIGTERM, prev)
    if rc != 0:
        print("bench.py: a rank failed (torch.distributed.run exit %d)" % rc, file=sys.stderr)
        return rc if rc > 0 else 1
    if len(lines) != 1:
        print("bench.py: expected one JSON line from rank 0, got %d" % len(lines), file=sys.stderr)
        return 3
    print(lines[0], flush=True)
    return 0


def _clock_under_load(device_index, run_step, sync, ms_per_step):
    """Shader clock while the workload runs: one extra, UNTIMED step with the
    libcordaprobe.so sampler resident beside it (8 one-wave workgroups, one per
    XCD, stamping s_memtime / s_memrealtime; corda_amd/csrc/clock_probe.hip).
    Returns the median per-interval clock and its spread."""
    import ctypes
    so = os.path.join(ROOT, "corda_amd", "libcordaprobe.so")
    if not os.path.exists(so):
        return {"error": "libcordaprobe.so not built"}
    lib = ctypes.CDLL(so)
    lib.cordaprobe_clock_start.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.POINTER(ctypes.c_void_p)]
    lib.cordaprobe_clock_finish.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_uint32,
                                            ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_double)]
    nblk, nsmp = 8, 65
    window = max(5.0, 0.7 * ms_per_step)  # inside the step: the sampler must not outlive the workload
    h = ctypes.c_void_p()
    rc = lib.cordaprobe_clock_start(device_index, window, nblk, nsmp, ctypes.byref(h))
    if rc not in (0, -2):
        return {"error": "cordaprobe_clock_start rc %d" % rc}
    run_step()
    sync()
    buf = (ctypes.c_double * (nblk * nsmp))()
    m = ctypes.c_uint32()
    mhz = ctypes.c_double()
    rc2 = lib.cordaprobe_clock_finish(h, buf, nblk * nsmp, ctypes.byref(m), ctypes.byref(mhz))
    if rc != 0 or rc2 != 0:
        return {"error": "sampler not resident before the step (rc %d) / finish rc %d" % (rc, rc2)}
    v = np.sort(np.array(buf[:m.value]))
    if v.size == 0:
        return {"error": "no samples"}
    return {"clock_ghz": float(np.median(v)), "clock_ghz_p10": float(np.percentile(v, 10)),
            "clock_ghz_p90": float(np.percentile(v, 90)), "samples": int(v.size), "window_ms": window,
            "realtime_mhz_check": mhz.value,
            "method": "s_memtime/s_memrealtime x 100 MHz per interval, 8 one-wave workgroups (one per XCD) "
                      "resident beside one extra untimed step of this workload; median over intervals"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--batch-log2", type=int, default=None, help="lanes per GPU (default 2^20 for c1, 2^24 otherwise)")
    ap.add_argument("--c4-txs", type=int, default=10_000_000 // 8)
    ap.add_argument("--native-leaves", action="store_true",
                    help="c4 / c4h: real-shaped cash-issue leaves from the native Kryo encoder (SURVEY 8f-4)")
    ap.add_argument("--components", action="store_true",
                    help="c4h: hand the library the transactions' Kryo components (cordahip_txcomp_submit); "
                         "the GPU writes the leaves")
    ap.add_argument("--device-encode", action="store_true",
                    help="c4: native leaves encoded on the GPU every step from the components in HBM "
                         "(cordahip_kryo_encode_device; implies --native-leaves)")
    ap.add_argument("--inflight", type=int, default=1,
                    help="c4h, c2h, c3h: calls outstanding at once (consecutive batches overlap on the device); "
                         "give --warmup >= K so every transaction set has grown its stages before timing")
    ap.add_argument("--cpu-sample", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-clock", action="store_true", help="skip the shader-clock sampling step")
    ap.add_argument("--global-log2", type=int, default=None,
                    help="C5 only: strong scaling over a fixed 2^G global batch (SURVEY 8d C5: G = 28)")
    args = ap.parse_args(argv)
    if args.inflight > 1 and args.warmup < args.inflight:
        # with fewer warmup calls than calls in flight, a transaction set would grow its
        # pinned stages (GBs of page-locked memory) inside the timed steps
        ap.error("--inflight %d needs --warmup >= %d" % (args.inflight, args.inflight))
    return args


def main():
    args = parse_args()
    if args.global_log2 and args.workload != "c5":
        raise SystemExit("bench.py: error: --global-log2 applies to --workload c5")
    if args.gpus < 1:
        raise SystemExit("bench.py: error: --gpus must be >= 1")
    if args.batch_log2 is None:
        args.batch_log2 = 20 if args.workload == "c1" else 24

    # --gpus N: one rank per GPU. Without a launcher's WORLD_SIZE, start the ranks
    # here (nothing has touched the GPU yet); under one, the two must agree.
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(_launch(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d" % (os.environ["WORLD_SIZE"], args.gpus), file=sys.stderr)
        sys.exit(2)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    stub = args.workload == "stub"

    # host threads next to the GPU, before HIP starts its own threads (they inherit it)
    from corda_amd.numa import bind_rank, numa_of_gpu
    _NUMA.update(bind_rank(local_rank, apply=not stub))
    if _NUMA.get("cpus_bound"):
        nodes = [numa_of_gpu(r) for r in range(local_world)]
        _NUMA["ranks_on_node"] = max(1, sum(1 for x in nodes if x and x["numa_node"] == _NUMA["numa_node"]))

    import torch
    import torch.distributed as dist
    from corda_amd.dist import gather_verdicts, max_over_ranks

    if stub:
        device = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
        sync = lambda: None  # noqa: E731
    else:
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("nccl", device_id=device)
        sync = lambda: torch.cuda.synchronize(device)  # noqa: E731
        try:  # the NUMA choice was made from sysfs before HIP init: confirm it names this device
            from corda_amd.numa import location_matches
            pr = torch.cuda.get_device_properties(local_rank)
            _NUMA["numa_check"] = location_matches(_NUMA, int(getattr(pr, "pci_bus_id", -1)),
                                                   int(getattr(pr, "pci_device_id", -1)),
                                                   int(getattr(pr, "pci_domain_id", 0)))
        except Exception as e:  # noqa: BLE001 - diagnostic only
            _NUMA["numa_check"] = "unavailable: %s" % type(e).__name__

    if stub:
        eng, stream = None, None
    else:
        from corda_amd.engine import Engine
        eng = Engine(1 << local_rank)
        # one explicit stream carries corpus generation, the kernels and the timing
        # events, so the events bracket exactly the launches they time
        stream = torch.cuda.Stream(device)
        torch.cuda.set_stream(stream)
    t_gen = time.perf_counter()
    wl = WORKLOADS[args.workload](eng, device, stream, rank, args)
    sync()
    t_gen = time.perf_counter() - t_gen
    host_timed = getattr(wl, "host_timed", False)

    def step(ev_s=None, ev_e=None):
        if ev_s is not None:
            ev_s.record(stream)
        wl.step()
        if ev_e is not None:
            ev_e.record(stream)
        verdict = getattr(wl, "verdict", None)
        if world > 1 and verdict is not None:
            gather_verdicts(verdict, world)  # the only data-path collective (RCCL all-gather)

    drain = getattr(wl, "drain", None)  # workloads with calls outstanding (c4h --inflight)

    def sync_all():
        if drain is not None:
            drain()
        sync()

    for _ in range(args.warmup):
        step()
    sync_all()
    if world > 1:
        dist.barrier()
    sync()
    evs = [(None, None)] * args.steps if host_timed else \
        [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(*evs[k])
    sync_all()  # every call the timed steps submitted has completed
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if host_timed:
        kernel_ms = elapsed * 1e3 / args.steps  # synchronous host-buffer drain: the wall clock is the measure
    else:
        kernel_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps

    # after the timed region: the verdict all-gather reassembles every rank's mask
    gather = None
    verdict = getattr(wl, "verdict", None)
    if world > 1 and verdict is not None:
        g = gather_verdicts(verdict, world)
        nv = verdict.numel()
        gather = bool(torch.equal(g[rank * nv:(rank + 1) * nv], verdict))
    # the shader clock this box holds under this workload (one more, untimed step)
    clock = None
    if not stub and not args.no_clock:
        clock = _clock_under_load(local_rank, step, sync_all, elapsed * 1e3 / args.steps)
    chk = wl.check()
    elapsed = max_over_ranks(elapsed, device)
    for key in ("mismatches_vs_construction", "mismatches_vs_oracle_open_lanes"):
        if key in chk:
            chk[key] = int(max_over_ranks(float(chk[key]), device))
    if gather is not None:
        chk["verdict_allgather_ok_all_ranks"] = max_over_ranks(0.0 if gather else 1.0, device) == 0.0
    numa_nodes = _gather_ints(_NUMA.get("numa_node"), world, device)

    if rank == 0:
        value = world * wl.units * args.steps / elapsed
        achieved = wl.macs * wl.units / (kernel_ms * 1e-3) / 1e12
        # HBM bytes per step from the committed PMC passes (tools/gpu_pmc.sh:
        # FETCH_SIZE and WRITE_SIZE in separate passes), scaled to this step
        traffic, traffic_src, traffic_fabric, traffic_kind = None, None, None, None
        traffic_hbm_modeled, valu_busy = None, None
        pmc_file = os.path.join(ROOT, "profiles", wl.pmc) if wl.pmc else None
        if pmc_file and os.path.exists(pmc_file):
            with open(pmc_file) as f:
                pmc = json.load(f)
            dv = pmc.get("total", {}).get("derived", {})
            if "valu_busy_est_4cyc" in dv:
                # VALU busy from the same PMC file: SQ_INSTS_VALU x the measured ~4 SIMD-cycles per
                # (VOP3-dominated) wave instruction / SIMD-cycles (SQ_ACTIVE_INST_VALU
                # counts issues on gfx950, so the issue fraction alone is the _issue figure)
                valu_busy = {"valu_busy": dv["valu_busy_est_4cyc"], "valu_busy_pmc_run": dv["valu_busy_est_4cyc"],
                             "valu_issue_frac": dv.get("valu_busy_direct"),
                             "valu_insts_per_unit": dv.get("valu_lane_insts_per_lane"),
                             "valu_wave_insts_per_unit": dv.get("valu_wave_insts_per_lane"),
                             "source": "profiles/%s total.derived (the verification kernels of one step)" % wl.pmc}
            per_unit = pmc.get("hbm_bytes_per_unit")
            traffic = per_unit * wl.units if per_unit else None
            traffic_src = "profiles/%s (bytes per unit x units per step)" % wl.pmc
            traffic_kind = ("measured: FETCH_SIZE/WRITE_SIZE counters (separate passes, FETCH_SIZE x2 per the gfx950 "
                            "correction), L2-to-fabric bytes = HBM + Infinity-Cache hits, an upper bound on HBM")
            if pmc.get("l2_fabric_bytes_per_unit"):
                # the counters stay primary; the HBM share is a model (tools/mall_sim.cpp, calibrated
                # on the same counters) and is reported under its own, explicit key
                traffic_hbm_modeled = traffic
                traffic = traffic_fabric = pmc["l2_fabric_bytes_per_unit"] * wl.units
                traffic_kind += ("; traffic_hbm_modeled: the ladder's Infinity-Cache hits removed by the calibrated "
                                 "model of tools/mall_sim.cpp (not a counter)")
            extra = getattr(wl, "extra_pmc", None)
            extra_file = os.path.join(ROOT, "profiles", extra[0]) if extra else None
            if traffic is not None and extra_file and os.path.exists(extra_file):
                with open(extra_file) as f:
                    xb = json.load(f)["l2_fabric_bytes_per_tx"] * extra[1]
                traffic += xb
                traffic_fabric = traffic_fabric + xb if traffic_fabric is not None else None
                traffic_hbm_modeled = traffic_hbm_modeled + xb if traffic_hbm_modeled is not None else None
                traffic_src += " + profiles/%s (the Kryo encoder kernels' L2-to-fabric bytes per tx x txs)" % extra[0]
                traffic_kind += "; the encoder's bytes added as read (no MALL split, an upper bound for its share)"
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "verifications/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if args.global_log2 else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": wl.data,
            "config": dict({"workload": wl.workload,
                            "parallelism": "dp%d (independent shards, RCCL all-gather of verdict masks)" % world,
                            "launcher": "torch.distributed.run (%s)" % ("bench.py child" if
                                                                        os.environ.get("CORDA_BENCH_CHILD") else
                                                                        "external") if world > 1 else "in-process",
                            "numa_node": _NUMA.get("numa_node"), "numa_nodes_by_rank": numa_nodes,
                            "numa": {k: v for k, v in _NUMA.items() if k != "numa_node"}},
                           **wl.config),
            "roofline": {"bound": "valu", "achieved": achieved, "peak": INT_MAC_PEAK_T,
                         "unit": "Tlimb-MAC/s", "frac": achieved / INT_MAC_PEAK_T, "traffic": traffic,
                         "traffic_source": traffic_src, "traffic_kind": traffic_kind,
                         "traffic_l2_fabric": traffic_fabric, "traffic_hbm_modeled": traffic_hbm_modeled,
                         "kernel": wl.kernel, "kernel_ms": kernel_ms,
                         "work_per_unit": "%d limb-MACs per verification (SURVEY §8d)" % wl.macs},
            "int_alu_peak_frac": achieved / INT_MAC_PEAK_T,
            "valu_busy": valu_busy,
            "verdict_check": chk,
            "corpus_gen_s": t_gen,
        }
        if eng is not None:
            # the library's device memory after the run (cordahip_device_mem): what this workload
            # held at its peak against the budget (CORDAHIP_DEVICE_MEM_BUDGET); torch's corpus
            # tensors are the caller's and not counted
            in_use, peak, budget = eng.device_mem(0)
            out["device_mem_gb"] = {"in_use": in_use / 1e9, "peak": peak / 1e9, "budget": budget / 1e9}
        ghz = clock.get("clock_ghz") if clock else None
        mpeak = 256 * MAD_U64_LANE_OPS_PER_CU_CYCLE * (ghz or 2.4) * 1e9 / 1e12
        out["roofline"]["peak_measured"] = mpeak
        out["roofline"]["peak_measured_basis"] = ("256 CU x %.2f v_mad_u64_u32 lane-ops/CU-cycle "
                                                  "(profiles/r01_int_rates.jsonl) x %s GHz" %
                                                  (MAD_U64_LANE_OPS_PER_CU_CYCLE, ("%.3f (clock_ghz)" % ghz) if ghz
                                                   else "2.4 (spec: no clock reading)"))
        out["roofline"]["frac_measured_peak"] = achieved / mpeak
        out["frac_measured_peak"] = achieved / mpeak
        if clock is not None:
            out["clock"] = clock
            if clock.get("clock_ghz"):
                out["clock_ghz"] = clock["clock_ghz"]
                # per-GPU verifications per 10^6 shader cycles: comparable across boxes
                out["verifs_per_mclk"] = value / world / (clock["clock_ghz"] * 1e3)
                vb = out.get("valu_busy")
                if vb and vb.get("valu_wave_insts_per_unit"):
                    # this run's VALU busy: the PMC file's wave instructions per unit x this step's
                    # units x ~4 SIMD-cycles each, over 1,024 SIMDs x this step's kernel time x the
                    # clock sampled under it. Under --pmc rocprofv3 runs dispatches one at a time, so
                    # the file's own figure (valu_busy_pmc_run) understates lines whose kernels
                    # overlap on several streams (the chunked and pipelined ones)
                    vb["valu_busy"] = (vb["valu_wave_insts_per_unit"] * wl.units * 4 /
                                       (1024 * kernel_ms * 1e-3 * clock["clock_ghz"] * 1e9))
                    vb["valu_busy_basis"] = ("PMC wave instructions per unit x units x 4 SIMD-cycles / "
                                             "(1024 SIMDs x kernel_ms x clock_ghz) of this run")
        if world == 1 and not args.no_cpu_baseline and not stub:
            # bounded samples sized for ~10 s of 16-thread CPU work each (C1: its whole 2^20 set)
            sample = args.cpu_sample or {"c1": 1 << 20, "c2": 1 << 22, "c3": 1 << 20, "c4": 1 << 20, "c5": 1 << 21,
                                         "c2h": 1 << 22, "c3h": 1 << 20, "c4h": 1 << 20}[args.workload]
            out["cpu_baseline"] = wl.cpu_baseline(min(sample, wl.units))
            out["cpu_baseline"].update(_cpu_info())
        print(json.dumps(out), flush=True)
    if eng is not None:
        eng.close()
    if world > 1:
        dist.destroy_process_group()


def _gather_ints(x, world, device):
    """Every rank's small int (None -> -1) as a list, for the rank-0 line."""
    if world == 1:
        return [x]
    import torch
    import torch.distributed as dist
    t = torch.tensor([-1 if x is None else int(x)], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [int(v[0]) for v in out]


if __name__ == "__main__":
    main()
