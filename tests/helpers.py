"""Shared builders for the parity tests: the same spec, GP data and hyperparameters feed the
HIP path (through the C ABI) and the CPU oracle (oracle/gpmpc_oracle.py)."""

from __future__ import annotations

import numpy as np

from gpmpc.models import get_spec
from gpmpc.synthetic import DEFAULT_HYPERS, initial_states, make_training_data
from oracle import gpmpc_oracle as O


def problem(name: str, n_train: int, seed: int = 1):
    spec = get_spec(name)
    data = make_training_data(spec, n_train, seed=seed)
    hyp = DEFAULT_HYPERS[name]
    return spec, data, hyp


def oracle_gps(data, hyp):
    return [O.ExactGP(X, y, *hyp[i]) for i, (X, y) in enumerate(data)]


def fitc_weights(gpp, M, seed=1337):
    """FITC (S, w) per GP from the product's restatement of `gpmpc/gpmpc.py:377-400` (pinned by
    tests/test_cpu_host.py::test_fitc_weights_match_reference_fixture)."""
    from gpmpc.gpmpc import GPMPC

    for gp in gpp:
        gp.K, gp.K_inv = gp.compute_covariances()
    me = type("Me", (), {})()
    me.gaussian_process = gpp
    me.np_random = np.random.default_rng(seed)
    return GPMPC.precompute_sparse_posterior_mean(me, M)


def fitc_oracle_gps(gpo, fitc):
    """Oracle GPs whose mean is the FITC approximation k(z, S) w; the variance stays exact."""
    for gp, (S, w) in zip(gpo, fitc):
        S = np.asarray(S, dtype=np.float64).reshape(len(w), -1)
        w = np.asarray(w, dtype=np.float64)

        def mean(Z, gp=gp, S=S, w=w):
            return O.se_kernel(np.atleast_2d(Z), S, gp.ell, gp.sf2) @ w

        def mean_grad(z, gp=gp, S=S, w=w):
            wv = O.se_kernel(z[None, :], S, gp.ell, gp.sf2)[0] * w
            return wv.sum(), (wv[:, None] * (S - z[None, :])).sum(0) / gp.ell**2

        gp.mean, gp.mean_grad = mean, mean_grad
    return gpo


def product_gps(data, hyp, device="cpu"):
    import torch

    from gpmpc.gp import GaussianProcess

    gps = []
    for i, (X, y) in enumerate(data):
        gp = GaussianProcess(torch.tensor(X), torch.tensor(y))
        gp.set_hyperparameters(*hyp[i])
        gps.append(gp)
    return gps


def lqr(spec):
    Q, R = np.diag(spec.q_diag), np.diag(spec.r_diag)
    dfdx, dfdu = spec.prior_jacobian(np.zeros(spec.nx), spec.u_eq)
    return O.setup_prior_dynamics(dfdx, dfdu, Q, R, spec.dt)


def oracle_step(spec, sol: O.SQPSolver, gps, x0, step, H, traj, prev, prob=0.95, tighten=True, uh=-1e-8, lqr_mats=None):
    """One reference select_action with the oracle: tightening from prev=(x_prev, u_prev) or None."""
    sd = spec.to_dict()
    nx, nu = spec.nx, spec.nu
    if tighten and prev is not None:
        Ad, Bd, K = lqr_mats
        sc, ic = O.propagate_constraint_limits(sd, gps, prev[0], prev[1], Ad, Bd, K, prob)
    else:
        sc, ic = np.zeros((2 * nx, H + 1)), np.zeros((2 * nu, H))
    lbx, ubx, lbu, ubu = O.stage_bounds(sd, sc, ic, uh)
    win = O.reference_window(traj, step, H)
    yref = np.zeros((H + 1, nx + nu))
    yref[:, :nx] = win.T
    yref[:H, nx:] = spec.u_eq
    st = sol.solve(x0, yref, lbx, ubx, lbu, ubu)
    return st, sc, ic


__all__ = ["problem", "oracle_gps", "product_gps", "fitc_weights", "fitc_oracle_gps", "lqr", "oracle_step",
           "initial_states", "O"]
