"""GP hyperparameter fit (`gpmpc/gp.py:49-69`): the fit oracle pinned by
closed forms and finite differences, and the product fit (exact_mll + autograd, the row-split
gradient of the data-parallel fit, Adam trajectories) against it on CPU tensors.  The same product
functions on the MI355X: tests/test_gpu_fit.py."""

import math

import numpy as np
import pytest
import scipy.stats

from oracle import gp_fit_oracle as F

# (model, GP index, N): d = 1 thrust GP, d = 3 pitch GP, d = 3 cartpole GP
CASES = [("quad2d", 0, 60), ("quad2d", 1, 80), ("cartpole", 1, 50)]
RAWS = [np.zeros(3), np.array([0.3, -0.7, -2.5]), np.array([-0.4, 1.1, -6.0])]


def case_data(name, i, n):
    from gpmpc.models import get_spec
    from gpmpc.synthetic import make_training_data

    return make_training_data(get_spec(name), n, seed=1)[i]


def product_gp(X, y, raw, device="cpu"):
    import torch

    from gpmpc.gp import GaussianProcess

    gp = GaussianProcess(torch.tensor(X, device=device), torch.tensor(y, device=device))
    for p, r in zip(gp.parameters(), raw):
        p.fill_(float(r))
    return gp


# ------------------------------------------------------------------ the oracle itself
def test_oracle_mll_closed_forms():
    # one training point: log N(y | 0, sf2 + noise)
    raw = np.array([0.2, -0.3, -1.0])
    ell, sf2, noise = F.constrained(raw)
    y = np.array([0.7])
    s = sf2 + noise
    want = -0.5 * y[0] ** 2 / s - 0.5 * math.log(s) - 0.5 * math.log(2 * math.pi)
    assert abs(F.mll(np.zeros((1, 2)), y, raw) - want) < 1e-14
    # scipy's multivariate normal log-density of K + noise I, divided by n
    X, y = case_data("quad2d", 1, 40)
    for raw in RAWS:
        ell, sf2, noise = F.constrained(raw)
        K = sf2 * np.exp(-0.5 * ((X[:, None] - X[None]) ** 2).sum(-1) / ell**2) + noise * np.eye(len(y))
        want = scipy.stats.multivariate_normal(mean=np.zeros(len(y)), cov=K).logpdf(y) / len(y)
        assert abs(F.mll(X, y, raw) - want) < 1e-10 * max(1.0, abs(want))


@pytest.mark.parametrize("name,i,n", CASES)
def test_oracle_gradient_matches_finite_differences(name, i, n):
    X, y = case_data(name, i, n)
    for raw in RAWS:
        val, g = F.mll_grad(X, y, raw)
        assert abs(val - F.mll(X, y, raw)) < 1e-11 * max(1.0, abs(val))
        h = 1e-5
        fd = np.array([(F.mll(X, y, raw + h * e) - F.mll(X, y, raw - h * e)) / (2 * h) for e in np.eye(3)])
        np.testing.assert_allclose(g, fd, rtol=1e-6, atol=1e-8 * (1 + np.abs(fd).max()))


def test_oracle_adam_matches_torch_adam():
    import torch

    rng = np.random.default_rng(4)
    grads = rng.standard_normal((25, 3)) * np.array([1.0, 1e-3, 30.0])
    p0 = rng.standard_normal(3)
    t = torch.tensor(p0.copy(), requires_grad=True)
    opt = torch.optim.Adam([t], lr=0.03)
    o = F.Adam(0.03)
    p = p0.copy()
    for g in grads:
        opt.zero_grad()
        t.grad = torch.tensor(g)
        opt.step()
        p = o.step(p, g)
        np.testing.assert_allclose(p, t.detach().numpy(), rtol=1e-13, atol=1e-15)


# ------------------------------------------------------------------ product vs oracle (CPU tensors)
def check_product_against_oracle(device):
    """Shared by this file (CPU) and tests/test_gpu_fit.py (cuda)."""
    import torch

    from gpmpc.distributed import mll_and_grad_partial
    from gpmpc.gp import exact_mll

    for name, i, n in CASES:
        X, y = case_data(name, i, n)
        for raw in RAWS:
            val, g = F.mll_grad(X, y, raw)
            gp = product_gp(X, y, raw, device)
            for p in gp.parameters():
                p.requires_grad_(True)
            m = exact_mll(gp)
            m.backward()
            ga = np.array([float(p.grad) for p in gp.parameters()])
            assert abs(float(m.detach()) - val) < 1e-11 * max(1.0, abs(val)), (name, i, raw)
            np.testing.assert_allclose(ga, g, rtol=1e-9, atol=1e-12 * (1 + np.abs(g).max()))
            # the data-parallel fit's row-split partials (two "ranks"), summed
            for p in gp.parameters():
                p.requires_grad_(False)
                p.grad = None
            with torch.no_grad():
                h = n // 2
                m0, g0 = mll_and_grad_partial(gp, slice(0, h))
                m1, g1 = mll_and_grad_partial(gp, slice(h, n))
            assert abs(float(m0) - val) < 1e-11 * max(1.0, abs(val)) and float(m0) == float(m1)
            np.testing.assert_allclose((g0 + g1).cpu().numpy(), g, rtol=1e-9, atol=1e-12 * (1 + np.abs(g).max()))


def check_fit_trajectories(device, steps=20, lr=0.02):
    from gpmpc.distributed import fit_gp_allreduce
    from gpmpc.gp import fit_gp

    for name, i, n in CASES:
        X, y = case_data(name, i, n)
        gp = product_gp(X, y, np.zeros(3), device)
        raw0 = np.array([float(p) for p in gp.parameters()])
        ref = F.fit(X, y, n_train=steps, lr=lr, raw0=raw0)
        assert ref["stop_margin"] > 1e-8, "early-stop comparison too close to its threshold to be decided"
        for fit in ("fit_gp", "fit_gp_allreduce"):
            gp = product_gp(X, y, raw0, device)
            hist = []
            if fit == "fit_gp":
                it = fit_gp(gp, n_train=steps, lr=lr, device=device, history=hist)
            else:
                it = fit_gp_allreduce(gp, n_train=steps, lr=lr, history=hist)
            assert it == ref["iters"] == len(hist), (name, i, fit)
            loss = np.array([h[0] for h in hist])
            raw = np.array([h[1] for h in hist])
            np.testing.assert_allclose(loss, ref["loss"], rtol=1e-8, atol=1e-12)
            np.testing.assert_allclose(raw, ref["raw"], rtol=1e-8, atol=1e-10)
            # K and K^-1 of the fitted GP (`gpmpc/gp.py:69`)
            ell, sf2, noise = F.constrained(ref["raw"][-1])
            K = sf2 * np.exp(-0.5 * ((X.reshape(n, -1)[:, None] - X.reshape(n, -1)[None]) ** 2).sum(-1) / ell**2)
            K += noise * np.eye(n)
            np.testing.assert_allclose(gp.K.cpu().numpy(), K, rtol=1e-7, atol=1e-12)
            assert gp.K.device.type == device


def check_early_stop(device):
    """A fit long enough to end on the reference's |dloss| < 1e-3 rule (`gpmpc/gp.py:65-66`):
    the product stops at the oracle's iteration with the oracle's parameters."""
    from gpmpc.gp import fit_gp

    X, y = case_data("quad2d", 0, 60)
    gp = product_gp(X, y, np.zeros(3), device)
    raw0 = np.array([float(p) for p in gp.parameters()])
    ref = F.fit(X, y, n_train=400, lr=0.1, raw0=raw0)
    assert ref["iters"] < 400 and ref["stop_margin"] > 1e-6
    hist = []
    it = fit_gp(gp, n_train=400, lr=0.1, device=device, history=hist)
    assert it == ref["iters"]
    np.testing.assert_allclose(np.array(hist[-1][1]), ref["raw"][-1], rtol=1e-7, atol=1e-9)


def test_product_fit_early_stop_matches_oracle_cpu():
    check_early_stop("cpu")


def test_product_mll_and_gradients_match_oracle_cpu():
    check_product_against_oracle("cpu")


def test_product_fit_trajectory_matches_oracle_cpu():
    check_fit_trajectories("cpu")
