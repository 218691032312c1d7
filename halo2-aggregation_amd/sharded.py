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


def points_fold(curve: int):
    """The fold every caller passes: the library's pm_points_sum over the
    gathered (world, 8) partials -- one host call and one inversion (round 5
    folded them with one pm_point_add ctypes call per rank)."""
    import halo2_amd as H

    return lambda rows: H.points_sum(curve, rows)


def start_gather(part, dist, device, world: int, out=None):
    """Enqueue the all-gather of this rank's affine partial (8 x u64) into one
    (world * 8) int64 tensor and return (work handle, tensor); finish_gather
    folds it.  One collective and one device-to-host copy per MSM (round 2:
    a copy per rank)."""
    import torch

    t = torch.from_numpy(np.ascontiguousarray(part, dtype=np.uint64).reshape(8).view(np.int64).copy()).to(device)
    if out is None:
        out = torch.empty(world * 8, dtype=torch.int64, device=device)
    work = dist.all_gather_into_tensor(out, t, async_op=True)
    return work, out


def finish_gather(pending, fold):
    """Wait for start_gather's collective and fold the partials in rank order
    (`fold(rows) -> 8 x u64`, rows the (world, 8) partials: points_fold)."""
    work, out = pending
    work.wait()
    rows = out.cpu().numpy().view(np.uint64).reshape(-1, 8)
    return np.asarray(fold(rows), dtype=np.uint64).reshape(8)


def combine_partials(part, dist, device, fold, world: int, gathered=None):
    """All-gather each rank's affine partial (8 x u64) and fold them with
    `fold(rows) -> 8 x u64` (points_fold).  Returns the full MSM result on
    every rank.  (`gathered`: an optional reusable (world * 8) int64 tensor.)"""
    part = np.ascontiguousarray(part, dtype=np.uint64).reshape(8)
    if world == 1:
        return part
    return finish_gather(start_gather(part, dist, device, world, gathered), fold)


class PartialPipe:
    """The exchange of MSM k overlapped with MSM k + 1: step(part) starts
    partial k's all-gather and folds partial k - 1's (returned), drain()
    folds the last one.  Every partial is gathered and folded; only the
    collective's latency moves behind the next MSM's kernels."""

    def __init__(self, dist, device, fold, world: int):
        import torch

        self.dist, self.device, self.fold, self.world = dist, device, fold, world
        self.bufs = [torch.empty(world * 8, dtype=torch.int64, device=device) for _ in range(2)]
        self.k = 0
        self.pending = None

    def step(self, part):
        if self.world == 1:
            return np.ascontiguousarray(part, dtype=np.uint64).reshape(8)
        nxt = start_gather(part, self.dist, self.device, self.world, self.bufs[self.k & 1])
        self.k += 1
        prev, self.pending = self.pending, nxt
        return finish_gather(prev, self.fold) if prev is not None else None

    def drain(self):
        if self.pending is None:
            return None
        prev, self.pending = self.pending, None
        return finish_gather(prev, self.fold)


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
