"""Multi-GPU layout of the batched GP-MPC path.

One process per GPU.  The B instances are independent, so they are sharded contiguously
across ranks and the control step has no collective.  The GP state is replicated: every
rank must hold bit-identical training data and hyperparameters, which
:func:`replicate_training_data` guarantees with one broadcast from rank 0 (RCCL over
xGMI on the GPUs, gloo on CPU).  Timing reductions (max over ranks) and statistics (sums)
are the only other collectives, outside the timed data path.
"""

from __future__ import annotations

import math

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


def shard_slice(global_batch: int, rank: int, world: int) -> range:
    """Global instance ids owned by ``rank`` when ``global_batch`` instances are split over
    ``world`` ranks (strong scaling, SURVEY.md §8(e) "contiguous B/G slices"): contiguous slices
    whose sizes differ by at most one, every instance on exactly one rank."""
    if global_batch < world:
        raise ValueError(f"global batch {global_batch} < {world} ranks")
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


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


def _coll_device():
    """Device of collective buffers: the current GPU for RCCL ("nccl"), the host for gloo."""
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_rows(a: np.ndarray) -> np.ndarray:
    """All-gather the rows of a 2-D array from every rank, concatenated in rank order (the same
    result on every rank).  Used once per learning epoch for the newly sampled transitions
    (the reference's single process stacks them at
    `scripts/run_gp_mpc.py:115-118`).  Row counts may differ between ranks."""
    a = np.ascontiguousarray(np.atleast_2d(np.asarray(a, dtype=np.float64)))
    rank, size = world()
    if size == 1:
        return a
    dev = _coll_device()
    n = torch.tensor([a.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(size)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    m = max(counts)
    buf = torch.zeros((m, a.shape[1]), dtype=torch.float64, device=dev)
    buf[: a.shape[0]] = torch.as_tensor(a, device=dev)
    parts = [torch.zeros_like(buf) for _ in range(size)]
    dist.all_gather(parts, buf)
    return np.concatenate([p[:c].cpu().numpy() for p, c in zip(parts, counts)], axis=0)


def assert_replicated(*arrays) -> None:
    """Raise if the arrays differ between ranks (order-sensitive checksum, max vs min over ranks).
    The data-parallel GP fit sums gradient row-slices and is only valid on identical data."""
    rank, size = world()
    if size == 1:
        return
    sig = []
    for a in arrays:
        v = np.asarray(a, dtype=np.float64).ravel()
        w = np.arange(1, v.size + 1, dtype=np.float64)
        sig += [float(v.size), float(v.sum()), float((w * v).sum()), float((v * v).sum())]
    dev = _coll_device()
    hi = torch.tensor(sig, dtype=torch.float64, device=dev)
    lo = -hi.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MAX)
    if not torch.equal(hi, -lo):
        raise RuntimeError("GP training data differs between ranks: the data-parallel fit needs identical "
                           "replicas (gather the transitions with gather_rows first)")


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


# ---------------------------------------------------------------------------- shared GP fit
def mll_and_grad_partial(gp, rows: slice | None = None):
    """Exact MLL / N (every rank, redundant Cholesky) and this rank's share of its gradient.

    d(MLL/N)/dθ = 1/(2N) tr((α αᵀ − K⁻¹) ∂K/∂θ) is split by ROWS of the trace: the rank sums
    rows ``rows`` of (α αᵀ − K⁻¹) ⊙ ∂K/∂θ for θ = (raw lengthscale, raw outputscale, raw noise)
    (softplus chain rule as gpytorch's constraints).  Summing the partials over ranks gives the
    full gradient (`gpmpc/gp.py:49-69` fits with gpytorch autograd).
    """
    from .gp import NOISE_LOWER

    X, y = gp.train_inputs[0], gp.train_targets
    n = X.shape[0]
    sp = torch.nn.functional.softplus
    ell, sf2 = sp(gp.raw_lengthscale), sp(gp.raw_outputscale)
    noise = sp(gp.raw_noise) + NOISE_LOWER
    d2 = torch.cdist(X, X).pow(2) if X.shape[1] > 1 else (X - X.T).pow(2)
    E = torch.exp(-0.5 * d2 / ell**2)
    K = sf2 * E + noise * torch.eye(n, dtype=X.dtype, device=X.device)
    L = torch.linalg.cholesky(K)
    a = torch.cholesky_solve(y[:, None], L)[:, 0]
    mll = (-0.5 * (y @ a) - torch.log(torch.diagonal(L)).sum() - 0.5 * n * math.log(2 * math.pi)) / n
    r = rows if rows is not None else slice(0, n)
    Kinv_r = torch.cholesky_solve(torch.eye(n, dtype=X.dtype, device=X.device)[:, r], L).T   # rows r of K^-1
    W = a[r, None] * a[None, :] - Kinv_r
    dK_dell = sf2 * E[r] * d2[r] / ell**3
    dK_dsf2 = E[r]
    idx = torch.arange(n, device=X.device)[r]
    g_ell = (W * dK_dell).sum()
    g_sf2 = (W * dK_dsf2).sum()
    g_noise = W[torch.arange(W.shape[0], device=X.device), idx].sum()      # dK/dnoise = I
    chain = torch.stack([torch.sigmoid(gp.raw_lengthscale), torch.sigmoid(gp.raw_outputscale),
                         torch.sigmoid(gp.raw_noise)])
    grad = 0.5 / n * torch.stack([g_ell, g_sf2, g_noise]) * chain
    return mll, grad


def fit_gp_allreduce(gp, n_train: int = 500, lr: float = 0.01, history: list | None = None) -> int:
    """Data-parallel Adam on −MLL (`gpmpc/gp.py:49-69`): each rank owns a contiguous row slice of
    the trace term, one all-reduce (sum) of the 3 gradient partials per iteration (RCCL over
    xGMI on the GPUs, gloo on CPU), every rank applies the same Adam step, so the replicas stay
    identical without a broadcast.  Early stop |Δloss| < 1e-3 like the reference.  Returns the
    number of Adam iterations; ``history`` as in :func:`gpmpc.gp.fit_gp`."""
    import math as _m

    rank, size = world()
    red_dev = None
    if size > 1 and dist.get_backend() == "nccl":   # RCCL reduces device tensors
        red_dev = torch.device("cuda", torch.cuda.current_device())
    n = gp.train_inputs[0].shape[0]
    per = _m.ceil(n / size)
    rows = slice(min(n, rank * per), min(n, (rank + 1) * per))
    params = gp.parameters()
    for p in params:
        p.requires_grad_(False)
    opt = torch.optim.Adam(params, lr=lr)
    last = _m.inf
    it = 0
    for it in range(1, n_train + 1):
        with torch.no_grad():
            mll, g = mll_and_grad_partial(gp, rows)
            if size > 1:
                gr = g.to(red_dev) if red_dev is not None else g
                dist.all_reduce(gr, op=dist.ReduceOp.SUM)
                g = gr.to(g.device)
        for p, gi in zip(params, g):
            p.grad = -gi.reshape(p.shape).clone()   # loss = -MLL
        opt.step()
        loss = -float(mll)
        if history is not None:
            history.append((loss, [float(p) for p in params]))
        if abs(last - loss) < 1e-3:
            break
        last = loss
    for p in params:
        p.grad = None
    gp._dev = None
    gp.K, gp.K_inv = gp.compute_covariances()
    return it
