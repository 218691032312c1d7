"""Multi-GPU sharding of the MSM: one process per GPU (torch.distributed).

The MSM shards by point slices: rank r of `world` owns pairs
[r*n_per_rank, (r+1)*n_per_rank) (the multi-GPU analogue of best_multiexp's
per-thread chunks).  The only exchange is an all-gather of one
affine partial point (64 B) per rank -- RCCL over xGMI under the "nccl" backend,
gloo in the CPU tests -- followed by an EC fold.  EC addition is not limb-wise,
so an all-reduce of limbs would be wrong.
"""
from __future__ import annotations

import numpy as np


def shard_range(rank: int, world: int, n_per_rank: int):
    """(first global index, count) of this rank's slice (weak scaling)."""
    return rank * n_per_rank, n_per_rank


def split_range(rank: int, world: int, n_total: int):
    """(first index, count) when a fixed n_total is split over ranks."""
    per = (n_total + world - 1) // world
    lo = min(n_total, rank * per)
    hi = min(n_total, lo + per)
    return lo, hi - lo


def combine_partials(part, dist, device, point_add, world: int, gathered=None):
    """All-gather each rank's affine partial (8 x u64) and fold them in rank
    order with `point_add(a, b) -> 8 x u64`.  Returns the full MSM result on
    every rank."""
    import torch

    part = np.ascontiguousarray(part, dtype=np.uint64).reshape(8)
    if world == 1:
        return part
    t = torch.from_numpy(part.view(np.int64).copy()).to(device)
    if gathered is None:
        gathered = [torch.zeros(8, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(gathered, t)
    acc = np.zeros(8, dtype=np.uint64)
    for g in gathered:
        acc = point_add(acc, g.cpu().numpy().view(np.uint64))
    return acc


def gather_batches(local, dist, world: int, gathered=None):
    """Accumulator batches: proofs are independent, so rank r
    owns its own B proofs and the only collective is an all-gather of the
    (B, 4, 8) accumulator points.  `local` is a torch tensor; returns the
    (world * B, 4, 8) tensor in rank order (the local tensor when world == 1)."""
    import torch

    if world == 1:
        return local
    if gathered is None:
        gathered = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(gathered, local)
    return torch.cat(gathered, dim=0)
