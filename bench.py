#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X Corda verification engine.

Workload (BASELINE.json configs[1], "C2"): one step = one pass of the hot path
(`Crypto.isValid(EDDSA_ED25519_SHA512, ...)` over a batch, kernel K1) over a
batch of 2^24 Ed25519 (key, sig, 32-byte txId) tuples resident in HBM, 1% of
them corrupted / non-canonical with SURVEY.md §8(d)'s fixed catalogue, plus
the RCCL all-gather of the per-GPU verdict bitmasks when N > 1.

Contract: `python bench.py --gpus N --steps K --warmup W` (N > 1 under
torch.distributed.run, one rank per GPU); rank 0 prints ONE JSON line.
Weak scaling: every rank verifies its own 2^24 batch; value = all ranks'
verifications / max-over-ranks wall time of the K timed steps.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "signature verifications/sec (whole node, 1/2/4/8 GPU) + % integer-ALU peak"
# algorithmic work per Ed25519 verification, in limb-MACs
# (32x32->64 multiply-accumulates of schoolbook radix-2^32: 64 per field mul).
LIMB_MACS_PER_ED25519 = 198_000
# Integer-ALU peak: 256 CUs x 64 v_mad_u64_u32 lane-ops per CU-cycle x 2.4 GHz
# (per-CU rate measured: profiles/r01_int_rates.jsonl, 59-62 lane-ops/CU-cycle).
INT_MAC_PEAK_T = 256 * 64 * 2.4e9 / 1e12


def cpu_baseline(pubs, sigs, msgs, sample: int):
    """Oracle (oracle/c, a C port of the i2p 0.2.0 path) on the box's host cores."""
    import ctypes
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import load_oracle  # oracle loader lives with the tests (checker only)

    orc = load_oracle()
    k = pubs[:sample].cpu().numpy().copy()
    s = sigs[:sample].cpu().numpy().copy()
    m = msgs[:sample].cpu().numpy().copy()
    out = np.zeros(sample, np.uint8)
    cores = max(1, min(16, os.cpu_count() or 1))
    t0 = time.perf_counter()
    orc.oracle_ed25519_verify_batch(sample, k.ctypes.data, s.ctypes.data, m.ctypes.data, 32, out.ctypes.data, cores)
    dt = time.perf_counter() - t0
    one = min(sample, 4096)
    out1 = np.zeros(one, np.uint8)
    t1 = time.perf_counter()
    orc.oracle_ed25519_verify_batch(one, k.ctypes.data, s.ctypes.data, m.ctypes.data, 32, out1.ctypes.data, 1)
    dt1 = time.perf_counter() - t1
    return {"value": sample / dt, "unit": "verifications/s", "cores": cores, "kind": "port",
            "sample": "first %d tuples of the rank-0 C2 batch (same corpus, 1%% corrupted), %d threads; "
                      "single-thread rate on %d tuples: %.0f/s" % (sample, cores, one, one / dt1),
            "single_thread_value": one / dt1, "wall_s": dt}, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch-log2", type=int, default=24)
    ap.add_argument("--cpu-sample", type=int, default=1 << 17)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)

    from corda_amd.corpus import make_c2_corpus
    from corda_amd.engine import Engine

    eng = Engine(1 << local_rank)
    # one explicit stream carries corpus generation, the kernel and the timing
    # events, so the events bracket exactly the launches they time
    stream = torch.cuda.Stream(device)
    torch.cuda.set_stream(stream)
    n = 1 << args.batch_log2
    t_gen = time.perf_counter()
    pubs, sigs, msgs, expected, cats = make_c2_corpus(eng, n, 0xC0DA0002 + rank, device, stream=stream)
    t_gen = time.perf_counter() - t_gen
    status = torch.empty(n, dtype=torch.uint8, device=device)
    verdict = torch.empty(n // 64, dtype=torch.int64, device=device)
    gathered = torch.empty(world * (n // 64), dtype=torch.int64, device=device) if world > 1 else None

    def step(ev_s=None, ev_e=None):
        if ev_s is not None:
            ev_s.record(stream)
        eng.ed25519_verify_device(pubs, sigs, msgs, status, verdict, device=0, stream=stream)
        if ev_e is not None:
            ev_e.record(stream)
        if world > 1:
            dist.all_gather_into_tensor(gathered, verdict)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(*evs[k])
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps

    # verdict sanity against the corpus construction (slide-dependent lanes excluded;
    # full bit-exact parity vs the oracle is tests/test_gpu_ed25519.py's job)
    known = expected >= 0
    mismatches = int((status[known].to(torch.int16) != expected[known]).sum())
    accepted = int((status == 0).sum())

    if world > 1:
        t = torch.tensor([elapsed, float(mismatches)], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
        mismatches = int(t[1])

    if rank == 0:
        value = world * n * args.steps / elapsed
        achieved = LIMB_MACS_PER_ED25519 * n / (kernel_ms * 1e-3) / 1e12
        traffic = None
        pmc_file = os.path.join(ROOT, "profiles", "r01_pmc_ed25519_verify.json")
        if os.path.exists(pmc_file):
            with open(pmc_file) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "verifications/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: seeded RFC 8032 tuples signed on the GPU (cordahip_ed25519_sign_device), "
                    "1% corrupted per SURVEY §8(d) C2",
            "config": {"workload": "C2: Ed25519 batch of 2^%d sigs per GPU, 32-byte txIds, 1%% corrupted/non-canonical"
                                   % args.batch_log2,
                       "batch_per_gpu": n, "msg_len": 32, "corrupt_frac": 0.01,
                       "parallelism": "dp%d (independent shards, RCCL all-gather of verdict masks)" % world},
            "roofline": {"bound": "valu", "achieved": achieved, "peak": INT_MAC_PEAK_T,
                         "unit": "Tlimb-MAC/s", "frac": achieved / INT_MAC_PEAK_T, "traffic": traffic,
                         "kernel": "ed25519_verify_kernel", "kernel_ms": kernel_ms,
                         "work_per_unit": "%d limb-MACs per verification (SURVEY §8d)" % LIMB_MACS_PER_ED25519},
            "int_alu_peak_frac": achieved / INT_MAC_PEAK_T,
            "verdict_check": {"mismatches_vs_construction": mismatches, "accepted": accepted,
                              "corrupted": int((expected != 0).sum())},
            "corpus_gen_s": t_gen,
        }
        if world == 1 and not args.no_cpu_baseline:
            cb, cpu_status = cpu_baseline(pubs, sigs, msgs, min(args.cpu_sample, n))
            cpu_mism = int((torch.from_numpy(cpu_status).to(device) != status[:len(cpu_status)]).sum())
            cb["gpu_vs_port_mismatches_on_sample"] = cpu_mism
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
