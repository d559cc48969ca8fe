"""Multi-GPU scoring: one process per GPU (torch.distributed backend "nccl" =
RCCL on ROCm; "gloo" for CPU tests).

* Batches: pairs sharded by contiguous blocks, per-pair int32 scores gathered
  to rank 0 over RCCL.  This is the north-star's "independent pairs shard
  across the GPUs of a node, RCCL only for the final score gather": no
  data-path collective, the only exchange is npairs int32 scores per step.
* One long pair (ColumnSlabs): the columns are cut into one
  slab per rank; slab edges travel GPU to GPU as tagged granules stored by the
  producing kernel into the next rank's IPC-mapped buffer, and the score is an
  all-reduce(MAX) of one int.

The reference has no multi-GPU path (no NCCL/MPI call
sites).
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


# ---- one pair split into column slabs -------------------------------

def slab_max(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-reduce(MAX) of the per-slab maxima: the pair's score, on every rank (RCCL;
    gloo reduces a host copy).  The only collective of the slab path."""
    if local.is_cuda and dist.get_backend(group) == "gloo":
        host = local.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.MAX, group=group)
        local.copy_(host)
        return local
    dist.all_reduce(local, op=dist.ReduceOp.MAX, group=group)
    return local


class ColumnSlabs:
    """One (seq1, seq2) pair split into column slabs, one per rank.

    Rank r scores columns [bounds[r], bounds[r+1]) of seq1 against all m rows of
    seq2 (lib: sw_score_slab_device).  The left edge of its slab -- H - G_INIT,
    E - G_EXT of the previous slab's last column, one tagged 16-byte granule per
    row -- is written straight into a buffer rank r owns by rank r-1's kernel,
    through an IPC mapping of that buffer (xGMI peer stores on a node): no host
    staging and no collective on the data path.  The ranks run as one wavefront
    pipeline; the only collective is slab_max, the all-reduce of one int.

    The all-reduce also orders launches: rank r's launch k+1 is queued behind
    it, so it cannot overwrite rank r+1's inflow before launch k there has read
    it; each launch tags its granules with a fresh epoch, common to all ranks."""

    def __init__(self, n: int, m: int, flags: int, group=None):
        from . import ipc_open, slab_alloc, slab_bounds
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.n, self.m, self.flags = n, m, flags
        self.bounds = slab_bounds(n, m, self.world, flags)
        self.inflow = slab_alloc(m) if self.rank > 0 else None
        handles = [None] * self.world
        dist.all_gather_object(handles, self.inflow.handle if self.inflow else None, group=group)
        self.outflow = ipc_open(handles[self.rank + 1]) if self.rank + 1 < self.world else 0
        self.epoch = 0
        self.score = torch.zeros(1, dtype=torch.int32, device="cuda")
        dist.barrier(group=group)   # every rank has mapped its outflow before any kernel runs

    @property
    def columns(self) -> tuple:
        return self.bounds[self.rank], self.bounds[self.rank + 1]

    def launch(self, d_arena_ptr: int, col_off: int, row_off: int, stream: Optional[int] = None) -> None:
        """Enqueue this rank's slab kernel (a fresh epoch) on `stream`; self.score then holds
        the slab's max.  The pair whose columns start at byte col_off and rows at row_off
        of the device arena."""
        from . import score_slab_device
        self.epoch += 1
        lo, hi = self.columns
        score_slab_device(d_arena_ptr, col_off + lo, hi - lo, row_off, self.m,
                          self.inflow.ptr if self.inflow else 0, self.outflow, self.epoch,
                          self.score.data_ptr(), self.flags, stream)

    def reduce(self) -> torch.Tensor:
        """The pair's score: all-reduce(MAX) of the slab maxima (1-int tensor, identical on
        every rank).  It also orders launches: rank r's next kernel is queued behind it."""
        return slab_max(self.score, self.group)

    def run(self, d_arena_ptr: int, col_off: int, row_off: int, stream: Optional[int] = None) -> torch.Tensor:
        """launch + reduce: score this rank's slab and return the pair's score."""
        self.launch(d_arena_ptr, col_off, row_off, stream)
        return self.reduce()

    def close(self) -> None:
        from . import ipc_close
        torch.cuda.synchronize()
        dist.barrier(group=self.group)   # no kernel still writes a buffer that is about to go
        if self.outflow:
            ipc_close(self.outflow)
            self.outflow = 0
        if self.inflow is not None:
            self.inflow.free()
            self.inflow = None
