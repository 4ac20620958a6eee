"""One process per GPU: rank environment, timestep partition, timing reduce.

Timesteps are independent (compute_optical_flow.py:162-177), so ranks share
nothing on the data path; the only collectives are the benchmark's barrier
and the max-over-ranks of its wall time (RCCL on GPUs, gloo on CPU tests).
"""
from __future__ import annotations

import os

from .solve import shard_ranges


def rank_env():
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def rank_k_range(rank: int, world: int, k0: int, k1: int):
    """Contiguous k-range [a, b) of ``rank`` when [k0, k1) is split over ``world``."""
    return shard_ranges(k0, k1, world)[rank]


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """Max of a float over all ranks (identity without a process group)."""
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, dist=None, device=None) -> float:
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return float(t.item())
