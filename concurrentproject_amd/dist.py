"""Multi-GPU batch scoring: one process per GPU, pairs sharded by contiguous
blocks, per-pair int32 scores gathered to rank 0 over RCCL (torch.distributed
backend "nccl" on ROCm; "gloo" for CPU tests).

The reference has no multi-GPU path (no NCCL/MPI call
sites); this is the north-star's "independent pairs shard across the GPUs of a
node, RCCL only for the final score gather".  There is no data-path collective:
each rank generates (or receives) its own shard and scores it locally; the
only exchange is npairs int32 scores per step.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch
import torch.distributed as dist


def shard_bounds(npairs: int, world: int, rank: int) -> tuple:
    """Contiguous block partition [lo, hi) of npairs over world ranks (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(npairs, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_scores(local: torch.Tensor, npairs: int, group=None) -> Optional[torch.Tensor]:
    """Gather every rank's int32 shard to rank 0 in global pair order.

    Shards may differ in length by one pair (shard_bounds); they are padded to
    the largest shard for the collective and trimmed afterwards.  Returns the
    full score vector on rank 0 and None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    width = shard_bounds(npairs, world, 0)[1]           # rank 0 holds the largest shard
    buf = torch.full((width,), -1, dtype=torch.int32, device=local.device)
    buf[: local.numel()] = local
    if rank == 0:
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.gather(buf, parts, dst=0, group=group)
        out = [p[: shard_bounds(npairs, world, r)[1] - shard_bounds(npairs, world, r)[0]] for r, p in enumerate(parts)]
        return torch.cat(out)
    dist.gather(buf, None, dst=0, group=group)
    return None


def score_sharded(npairs: int, score_shard: Callable[[int, int], Sequence[int]], device: str = "cpu",
                  group=None) -> Optional[list]:
    """Score pairs [lo, hi) of this rank with ``score_shard(lo, hi)`` and gather all
    scores to rank 0 (returns the list there, None elsewhere)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_bounds(npairs, world, rank)
    local = torch.tensor(list(score_shard(lo, hi)), dtype=torch.int32, device=device)
    full = gather_scores(local, npairs, group)
    return None if full is None else full.cpu().tolist()
