"""Env-level data parallelism across GPUs.

Envs are independent: rank r owns a contiguous block of global env ids and seeds
env g with ``base_seed + g``, so a sharded run is bit-identical to the same envs run
on one GPU.  There is no collective on the step; the only cross-rank traffic is the
timing / metric reduction after the timed region (one tiny all_reduce).
"""
from __future__ import annotations

import os


def world() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def shard(global_envs: int, rank: int, world_size: int) -> tuple[int, int]:
    """Strong scaling: (offset, count) of rank's contiguous block of `global_envs`."""
    if not 0 <= rank < world_size:
        raise ValueError("rank out of range")
    base, rem = divmod(global_envs, world_size)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def weak_shard(envs_per_rank: int, rank: int) -> tuple[int, int]:
    """Weak scaling: every rank owns `envs_per_rank` envs, ids [rank*E, (rank+1)*E)."""
    return rank * envs_per_rank, envs_per_rank


def env_seeds(base_seed: int, offset: int, count: int) -> list[int]:
    return [int(base_seed) + offset + e for e in range(count)]


def max_over_ranks(value: float, device=None) -> float:
    """MAX of a scalar over ranks (the bench's elapsed time); identity when not distributed."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device=None) -> float:
    """SUM of a scalar over ranks (the intersection bench's live-vehicle count); identity when not
    distributed."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
