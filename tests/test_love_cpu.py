"""LOVE variance (gpytorch ``fast_pred_var``, the reference's tightening variance,
`gpmpc/gpmpc.py:442-444`): the host Lanczos root against the numpy restatement and the exact
variance.  gpytorch is absent here, so the restatement is unpinned; these tests pin the root's
algebra (R^T K R = I on the Krylov space; the full-rank root gives the exact variance)."""

import numpy as np
import pytest
import torch

from helpers import O, problem


def _gp(name, N, g=0):
    from gpmpc.gp import GaussianProcess
    from gpmpc.synthetic import DEFAULT_HYPERS

    spec, data, hyp = problem(name, N)
    X, y = data[g]
    gp = GaussianProcess(torch.tensor(X), torch.tensor(y))
    gp.set_hyperparameters(*DEFAULT_HYPERS[spec.name][g])
    return gp, O.ExactGP(X, y, *hyp[g])


@pytest.mark.parametrize("N,rank", [(60, 100), (200, 100), (300, 40)])
def test_love_root_is_a_krylov_inverse_root(N, rank):
    gp, og = _gp("quad2d", N)
    R = gp.love_root(rank).numpy()
    K = gp.K.numpy()
    assert R.shape[0] == N and R.shape[1] <= min(rank, N)
    np.testing.assert_allclose(R.T @ K @ R, np.eye(R.shape[1]), atol=1e-8)


def test_love_root_matches_numpy_restatement():
    gp, og = _gp("quad2d", 200)
    gen = torch.Generator(device="cpu").manual_seed(0)
    start = torch.randn(200, dtype=torch.float64, generator=gen).numpy()
    R_t = gp.love_root(50, seed=0).numpy()
    R_o = O.lanczos_love_root(gp.K.numpy(), 50, start)   # same K: the algorithm, not the kernel rounding
    assert R_t.shape == R_o.shape
    # the roots agree where they are used: the predictive variance (R R^T itself is ill-conditioned,
    # cond(K) ~ 4e7 here)
    Z = np.random.default_rng(5).normal(scale=0.5, size=(64, og.X.shape[1]))
    v_t, v_o = O.love_var(og, R_t, Z), O.love_var(og, R_o, Z)
    np.testing.assert_allclose(v_t, v_o, rtol=0, atol=1e-9 * og.sf2)


@pytest.mark.parametrize("N", [60, 200, 1000])
def test_love_variance_bounds_the_exact_variance(N):
    """R R^T = Q T^-1 Q^T is the inverse of K projected on the Krylov space, so it is below
    K^-1 in the Loewner order: the LOVE variance is never below the exact one (up to rounding),
    and for these smooth kernels it is within 0.1 % of it."""
    gp, og = _gp("quad2d", N)
    R = gp.love_root(100).numpy()
    rng = np.random.default_rng(1)
    Z = og.X[rng.integers(0, N, 50)] + rng.normal(scale=0.1, size=(50, og.X.shape[1]))
    ve, vl = og.var(Z), O.love_var(og, R, Z)
    assert (vl - ve).min() >= -1e-11 * og.sf2
    np.testing.assert_allclose(vl, ve, rtol=1e-3, atol=1e-10 * og.sf2)


def test_love_threshold_follows_gpytorch_cholesky_size():
    from gpmpc.gp import LOVE_CHOLESKY_ROWS

    assert LOVE_CHOLESKY_ROWS == 800   # gpytorch.settings.max_cholesky_size default


def test_default_tightening_variance_is_the_references_fast_pred_var():
    """GPMPC and bench.py default to variance='love': the reference's propagate_constraint_limits
    runs under gpytorch.settings.fast_pred_var() (gpmpc/gpmpc.py:442-444), i.e. exact up to 800
    training rows (BatchSolver applies the Lanczos root only above LOVE_CHOLESKY_ROWS)."""
    import inspect
    import sys
    from pathlib import Path

    from gpmpc.gpmpc import GPMPC
    from gpmpc.models import get_spec

    assert inspect.signature(GPMPC.__init__).parameters["variance"].default == "love"
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    assert bench.parse_args([]).variance == "love"
    assert "LOVE" not in bench.workload_name(get_spec("quad2d"), bench.parse_args([]))   # N = 200: exact
    assert "LOVE" in bench.workload_name(get_spec("quad2d"), bench.parse_args(["--n-train", "1000"]))
