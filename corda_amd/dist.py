"""Multi-GPU plumbing: one process per GPU, torch.distributed over RCCL.

SURVEY.md §8(e): signature verifications are independent units, so a batch
shards into contiguous 64-aligned index ranges (one per rank) with no
data-path collective; the only exchange is ONE all-gather of the per-rank
verdict bitmasks (RCCL over xGMI on MI355X; gloo in the CPU tests).
"""
from __future__ import annotations

from typing import Tuple


def shard_range(n: int, rank: int, world: int, align: int = 64) -> Tuple[int, int]:
    """Contiguous [lo, hi) of n units for `rank`; shard starts are `align`-aligned so every
    rank's verdict words cover whole 64-lane groups and concatenate without shifting."""
    per = ((n + world - 1) // world + align - 1) // align * align
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def gather_verdicts(verdict_words, world: int, group=None):
    """All-gather every rank's int64 verdict words (same length on every rank) into one tensor."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return verdict_words
    out = torch.empty(world * verdict_words.numel(), dtype=verdict_words.dtype, device=verdict_words.device)
    dist.all_gather_into_tensor(out, verdict_words.contiguous(), group=group)
    return out


def max_over_ranks(x: float, device=None) -> float:
    """The job's time is the slowest rank's time (bench contract)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])
