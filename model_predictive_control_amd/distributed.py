"""Multi-GPU sharding of the batched MPC solve (one process per GPU).

Every x0 instance is independent, so a batch is split
into contiguous shards, one per rank, and solved with no communication on the
solve path.  The only collective is the optional final gather of the input
trajectories to every rank (RCCL all-gather over xGMI on GPUs; gloo on CPU in
tests), done outside any timed region.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), \
        int(os.environ.get("LOCAL_RANK", 0))


def shard_bounds(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) slice of ``total`` instances owned by ``rank``."""
    q, r = divmod(total, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def shard(t: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    lo, hi = shard_bounds(t.shape[0], rank, world)
    return t[lo:hi]


def gather_shards(local: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """All-gather equal-or-ragged contiguous shards back into (total, ...)."""
    world = dist.get_world_size(group)
    sizes = [shard_bounds(total, r, world) for r in range(world)]
    cap = max(hi - lo for lo, hi in sizes)
    pad = local.new_zeros((cap,) + tuple(local.shape[1:]))
    pad[: local.shape[0]] = local
    out = local.new_empty((world * cap,) + tuple(local.shape[1:]))
    dist.all_gather_into_tensor(out, pad.contiguous(), group=group)
    parts = [out[r * cap: r * cap + (hi - lo)] for r, (lo, hi) in enumerate(sizes)]
    return torch.cat(parts, 0)


def max_over_ranks(value: float, device) -> float:
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device) -> float:
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
