"""Multi-GPU layout of the batched GP-MPC path.

One process per GPU.  The B instances are independent, so they are sharded contiguously
across ranks and the control step has no collective.  The GP state is replicated: every
rank must hold bit-identical training data and hyperparameters, which
:func:`replicate_training_data` guarantees with one broadcast from rank 0 (RCCL over
xGMI on the GPUs, gloo on CPU).  Timing reductions (max over ranks) and statistics (sums)
are the only other collectives, outside the timed data path.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def world() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(batch_per_rank: int, rank: int) -> range:
    """Global instance ids owned by ``rank`` (weak scaling: a fixed batch per rank)."""
    return range(rank * batch_per_rank, (rank + 1) * batch_per_rank)


def replicate_training_data(data: list[tuple[np.ndarray, np.ndarray]], device=None) -> list[tuple[np.ndarray, np.ndarray]]:
    """Broadcast every GP's (X, y) from rank 0 so all replicas are identical."""
    rank, size = world()
    if size == 1:
        return data
    out = []
    for X, y in data:
        dev = device if device is not None else torch.device("cpu")
        xt = torch.as_tensor(np.ascontiguousarray(X), dtype=torch.float64, device=dev).clone()
        yt = torch.as_tensor(np.ascontiguousarray(y), dtype=torch.float64, device=dev).clone()
        dist.broadcast(xt, src=0)
        dist.broadcast(yt, src=0)
        out.append((xt.cpu().numpy(), yt.cpu().numpy()))
    return out


def max_over_ranks(values: list[float], device=None) -> list[float]:
    rank, size = world()
    if size == 1:
        return list(values)
    t = torch.tensor(values, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


def sum_over_ranks(t: torch.Tensor) -> torch.Tensor:
    rank, size = world()
    if size > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t
