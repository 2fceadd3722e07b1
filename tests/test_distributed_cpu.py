"""world_size-2 gloo test of the sharding / replication / reduction logic used by bench.py."""

import os
import socket
import sys
from pathlib import Path

import numpy as np
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    sys.path[:0] = [str(ROOT / "gp-mpc_amd"), str(ROOT)]
    import torch
    import torch.distributed as dist

    from gpmpc import distributed as D
    from gpmpc.models import get_spec
    from gpmpc.synthetic import initial_states, make_training_data

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = get_spec("quad2d")
    # rank 1 starts from a different seed: replication must overwrite it with rank 0's data
    data = make_training_data(spec, 16, seed=1 if rank == 0 else 99)
    rep = D.replicate_training_data(data)
    ids = list(D.shard_range(8, rank))
    x0, ph = initial_states(spec, spec.reference_trajectory(), 8 * world)
    mine = torch.tensor(ph[ids[0]:ids[-1] + 1], dtype=torch.int64)
    gathered = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    t = D.max_over_ranks([float(rank + 1), 1.0])
    s = D.sum_over_ranks(torch.ones(3, dtype=torch.float64))
    out.put((rank, [x.tolist() for x, _ in rep], [y.tolist() for _, y in rep], torch.cat(gathered).tolist(), t,
             s.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_and_replication():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, x0, y0, g0, t0, s0), (_, x1, y1, g1, t1, s1) = res
    assert x0 == x1 and y0 == y1                       # GP replicas identical after the broadcast
    assert g0 == g1 == list(range(16))                 # 2 x 8 instances, contiguous, no overlap
    assert t0 == t1 == [2.0, 1.0]                      # max over ranks
    assert s0 == s1 == [2.0, 2.0, 2.0]
    from gpmpc.models import get_spec
    from gpmpc.synthetic import make_training_data

    ref = make_training_data(get_spec("quad2d"), 16, seed=1)
    np.testing.assert_array_equal(np.array(x0[0]), ref[0][0])


def _fit_worker(rank, world, port, out):
    sys.path[:0] = [str(ROOT / "gp-mpc_amd"), str(ROOT)]
    import torch
    import torch.distributed as dist

    from gpmpc import distributed as D
    from gpmpc.gp import GaussianProcess
    from gpmpc.models import get_spec
    from gpmpc.synthetic import make_training_data

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, y = make_training_data(get_spec("quad2d"), 60, seed=1)[1]
    gp = GaussianProcess(torch.tensor(X), torch.tensor(y))
    it = D.fit_gp_allreduce(gp, n_train=40, lr=0.05)
    out.put((rank, it, gp.lengthscale, gp.outputscale, gp.noise))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gp_fit_allreduce_matches_single_process():
    """row-split MLL gradient + all-reduce == the single-process autograd fit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fit_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1:] == res[1][1:]            # replicas bit-identical without a broadcast
    sys.path[:0] = [str(ROOT / "gp-mpc_amd")]
    import torch

    from gpmpc.gp import GaussianProcess, fit_gp
    from gpmpc.models import get_spec
    from gpmpc.synthetic import make_training_data

    X, y = make_training_data(get_spec("quad2d"), 60, seed=1)[1]
    ref = GaussianProcess(torch.tensor(X), torch.tensor(y))
    fit_gp(ref, n_train=40, lr=0.05)
    np.testing.assert_allclose(res[0][2:], [ref.lengthscale, ref.outputscale, ref.noise], rtol=1e-8)


def _gather_worker(rank, world, port, out):
    sys.path[:0] = [str(ROOT / "gp-mpc_amd"), str(ROOT)]
    import torch
    import torch.distributed as dist

    from gpmpc import distributed as D
    from gpmpc.gp import GaussianProcess

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # each rank sampled its own transitions (different counts too): learning.learn gathers them
    rng = np.random.default_rng([5, rank])
    n = 12 + 3 * rank
    inputs = rng.uniform(-1, 1, size=(n, 3))
    targets = np.sin(2 * inputs[:, :1]) + 0.01 * rng.standard_normal((n, 1))
    x_train, y_train = D.gather_rows(inputs), D.gather_rows(targets)
    D.assert_replicated(x_train, y_train)          # identical replicas: no error
    try:
        D.assert_replicated(inputs)                # rank-local data: must be refused
        refused = False
    except RuntimeError:
        refused = True
    gp = GaussianProcess(torch.tensor(x_train), torch.tensor(y_train[:, 0]))
    it = D.fit_gp_allreduce(gp, n_train=30, lr=0.05)
    out.put((rank, x_train.tolist(), y_train.tolist(), refused, it, gp.lengthscale, gp.outputscale, gp.noise))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_learning_epoch_gathers_transitions_before_the_fit():
    """per-epoch all-gather of the newly sampled transitions, so both ranks fit
    identical GPs on identical x_train (gpmpc/learning.py learn; `scripts/run_gp_mpc.py:115-120`)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0, r1 = res
    assert r0[1] == r1[1] and r0[2] == r1[2]                 # identical x_train / y_train
    assert len(r0[1]) == 12 + 15                             # rank 0's 12 rows then rank 1's 15
    rng0 = np.random.default_rng([5, 0])
    np.testing.assert_array_equal(np.array(r0[1][:12]), rng0.uniform(-1, 1, size=(12, 3)))
    assert r0[3] and r1[3]                                   # rank-local data is refused
    assert r0[4:] == r1[4:]                                  # identical fitted hyperparameters
    sys.path[:0] = [str(ROOT / "gp-mpc_amd")]
    import torch

    from gpmpc.gp import GaussianProcess, fit_gp

    ref = GaussianProcess(torch.tensor(np.array(r0[1])), torch.tensor(np.array(r0[2])[:, 0]))
    fit_gp(ref, n_train=30, lr=0.05)
    np.testing.assert_allclose(r0[5:], [ref.lengthscale, ref.outputscale, ref.noise], rtol=1e-8)
