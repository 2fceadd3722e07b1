"""Generate golden vectors by running the REFERENCE's own functions (this container only).

The reference (`/root/reference/gpmpc`) imports casadi, gpytorch and acados_template,
none of which is installed.  This script registers minimal stand-in
modules for those three names, imports `gpmpc.gp` and `gpmpc.gpmpc` from
`/root/reference`, and runs the reference functions that are pure numpy/scipy/torch once
their inputs exist:

  covSE_single, covSE_vectorized         gpmpc/gp.py:12-21     (casadi stand-in: numpy)
  GaussianProcess.compute_covariances    gpmpc/gp.py:43-46     (gpytorch stand-in: exact GP)
  gpytorch_predict2casadi                gpmpc/gp.py:72-85     (casadi stand-in evaluates eagerly)
  GPMPC.propagate_constraint_limits      gpmpc/gpmpc.py:425-498
  GPMPC.precompute_sparse_posterior_mean gpmpc/gpmpc.py:377-400
  GPMPC.setup_prior_dynamics             gpmpc/gpmpc.py:500-507 (+ discretize_linear_system)
  GPMPC.reference_trajectory             gpmpc/gpmpc.py:509-514
  GPMPC.setup_constraints                gpmpc/gpmpc.py:327-332

The gpytorch stand-in implements the EXACT GP posterior (the reference runs under
``fast_pred_var`` -- LOVE -- whose approximation is not reproduced).
Only the inputs and outputs are saved (``golden_quad3d.npz``); nothing of the reference is
copied.  Re-run:  python tests/golden/make_golden.py
"""

from __future__ import annotations

import contextlib
import sys
import types
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]


# --------------------------------------------------------------------------- stand-ins
class _Eager:
    """casadi stand-in: symbols are bound to concrete numpy values at creation."""

    bind: dict = {}

    @staticmethod
    def sym(name, *shape):
        v = _Eager.bind.get(name)
        if v is None:
            v = np.zeros(shape if len(shape) > 1 else (shape[0], 1))
        return np.asarray(v, dtype=np.float64).reshape(shape if len(shape) > 1 else (shape[0], 1))


class _Function:
    def __init__(self, name, ins, outs, in_names=None, out_names=None):
        self.outs = outs
        self.out_names = out_names

    def __call__(self, *args, **kwargs):
        if self.out_names is not None:
            return {n: o for n, o in zip(self.out_names, self.outs)}
        return self.outs[0]


def _install_stubs():
    cs = types.ModuleType("casadi")
    cs.sum1 = lambda a: np.sum(a, axis=0, keepdims=True)
    cs.sum2 = lambda a: np.sum(a, axis=1, keepdims=True)
    cs.exp = np.exp
    cs.repmat = lambda a, r, c: np.tile(a, (r, c))
    cs.SX = types.SimpleNamespace(sym=_Eager.sym)
    cs.MX = types.SimpleNamespace(sym=_Eager.sym)
    cs.Function = _Function
    cs.vertcat = lambda *a: np.vstack([np.atleast_2d(x).reshape(-1, 1) for x in a])
    sys.modules["casadi"] = cs

    at = types.ModuleType("acados_template")
    for n in ("AcadosModel", "AcadosOcp", "AcadosOcpSolver"):
        setattr(at, n, type(n, (), {}))
    sys.modules["acados_template"] = at

    gp = types.ModuleType("gpytorch")

    class _Lazy:
        def __init__(self, t):
            self.t = t

        def to_dense(self):
            return self.t

        def add_diag(self, d):
            return _Lazy(self.t + torch.eye(self.t.shape[0], dtype=self.t.dtype) * d)

    class RBFKernel:
        def __init__(self):
            self.lengthscale = torch.ones(1, 1, dtype=torch.float64)

    class ScaleKernel:
        def __init__(self, base):
            self.base_kernel = base
            self.outputscale = torch.tensor(1.0, dtype=torch.float64)

        def __call__(self, a, b=None):
            b = a if b is None else b
            ell = self.base_kernel.lengthscale.reshape(())
            d2 = ((a[:, None, :] - b[None, :, :]) ** 2).sum(-1)
            return _Lazy(self.outputscale * torch.exp(-0.5 * d2 / ell**2))

    class MultivariateNormal:
        def __init__(self, mean, cov):
            self.mean = mean
            self.covariance_matrix = cov.to_dense() if isinstance(cov, _Lazy) else cov

    class GaussianLikelihood:
        def __init__(self, noise_constraint=None):
            self.noise = torch.tensor([1e-4], dtype=torch.float64)

        def __call__(self, mvn):
            n = mvn.covariance_matrix.shape[0]
            return MultivariateNormal(mvn.mean, mvn.covariance_matrix + self.noise * torch.eye(n, dtype=torch.float64))

    class ExactGP:
        def __init__(self, x, y, likelihood):
            self.train_inputs = (x,)
            self.train_targets = y
            self.likelihood = likelihood
            self.training = True

        def eval(self):
            self.training = False
            return self

        def __call__(self, x):  # exact posterior in eval mode
            X, y = self.train_inputs[0], self.train_targets
            Kxx = self.covar_module(X).add_diag(self.likelihood.noise).to_dense()
            Kzx = self.covar_module(x, X).to_dense()
            Kzz = self.covar_module(x).to_dense()
            sol = torch.linalg.solve(Kxx, Kzx.T)
            return MultivariateNormal(Kzx @ torch.linalg.solve(Kxx, y), Kzz - Kzx @ sol)

    gp.models = types.SimpleNamespace(ExactGP=ExactGP)
    gp.constraints = types.SimpleNamespace(GreaterThan=lambda v: v)
    gp.mlls = types.SimpleNamespace()
    sys.modules["gpytorch"] = gp
    for sub, attrs in {
        "gpytorch.distributions": dict(MultivariateNormal=MultivariateNormal),
        "gpytorch.kernels": dict(RBFKernel=RBFKernel, ScaleKernel=ScaleKernel),
        "gpytorch.likelihoods": dict(GaussianLikelihood=GaussianLikelihood),
        "gpytorch.means": dict(ZeroMean=lambda: None),
        "gpytorch.settings": dict(fast_pred_var=lambda state=True: contextlib.nullcontext(),
                                  fast_pred_samples=lambda state=True: contextlib.nullcontext()),
    }.items():
        m = types.ModuleType(sub)
        m.__dict__.update(attrs)
        sys.modules[sub] = m


def main():
    sys.path.insert(0, str(REPO / "gp-mpc_amd"))
    from gpmpc.models import quad3d_spec  # noqa: E402  (the build's spec: numbers only)

    _install_stubs()
    sys.path.insert(0, str(REF))

    # the reference package shadows the build's package name from here on
    for k in [k for k in sys.modules if k == "gpmpc" or k.startswith("gpmpc.")]:
        del sys.modules[k]
    sys.path.remove(str(REPO / "gp-mpc_amd"))
    import gpmpc.gp as rgp  # noqa: E402
    import gpmpc.gpmpc as rgpmpc  # noqa: E402

    assert Path(rgp.__file__).resolve().is_relative_to(REF), rgp.__file__
    spec = quad3d_spec()
    rng = np.random.default_rng(1234)
    out = {}

    # ---- a1/a2: SE kernels --------------------------------------------------------
    X = rng.uniform(-1, 1, (17, 3))
    z = rng.uniform(-1, 1, 3)
    ell, sf2 = 0.7, 1.3
    out["k_X"], out["k_z"], out["k_ell"], out["k_sf2"] = X, z, ell, sf2
    out["k_single"] = np.asarray(rgp.covSE_single(z.reshape(3, 1), X.T, ell, sf2)).ravel()
    out["k_vec"] = np.asarray(rgp.covSE_vectorized(z.reshape(3, 1), X, ell, sf2)).ravel()

    # ---- a3/a5: GaussianProcess K, K_inv and the casadi mean export ---------------
    N = 40
    hyp = [(0.2, 25.0, 1e-4), (2.0, 50.0, 2e-4), (1.5, 40.0, 3e-4)]
    gp_idx = [[0], [1, 2, 3], [4, 5, 6]]
    Xtr = np.column_stack([rng.uniform(0.12, 0.59, N), rng.uniform(-0.6, 0.6, N), rng.uniform(-3, 3, N),
                           rng.uniform(-0.43, 0.43, N), rng.uniform(-0.6, 0.6, N), rng.uniform(-3, 3, N),
                           rng.uniform(-0.43, 0.43, N)])
    Ytr = np.column_stack([8.8 * Xtr[:, 0] + 1.8, -14.4 * Xtr[:, 1] - 1.5 * Xtr[:, 2] + 8.0 * Xtr[:, 3],
                           -14.4 * Xtr[:, 4] - 1.5 * Xtr[:, 5] + 8.0 * Xtr[:, 6]]) + 0.01 * rng.standard_normal((N, 3))
    gps = []
    for i, idx in enumerate(gp_idx):
        g = rgp.GaussianProcess(torch.tensor(Xtr[:, idx]), torch.tensor(Ytr[:, i]))
        g.covar_module.base_kernel.lengthscale = torch.tensor([[hyp[i][0]]], dtype=torch.float64)
        g.covar_module.outputscale = torch.tensor(hyp[i][1], dtype=torch.float64)
        g.likelihood.noise = torch.tensor([hyp[i][2]], dtype=torch.float64)
        g.K, g.K_inv = g.compute_covariances()
        gps.append(g)
        out[f"gp{i}_K"] = g.K.numpy()
        out[f"gp{i}_Kinv"] = g.K_inv.numpy()
    out["gp_Xtr"], out["gp_Ytr"], out["gp_hyp"] = Xtr, Ytr, np.array(hyp)
    Zq = np.column_stack([rng.uniform(0.1, 0.6, 9), rng.uniform(-0.7, 0.7, 9), rng.uniform(-3, 3, 9),
                          rng.uniform(-0.5, 0.5, 9), rng.uniform(-0.7, 0.7, 9), rng.uniform(-3, 3, 9),
                          rng.uniform(-0.5, 0.5, 9)])
    out["gp_Zq"] = Zq
    for i, idx in enumerate(gp_idx):
        means = []
        for q in range(Zq.shape[0]):
            _Eager.bind = {"z": Zq[q, idx]}
            means.append(float(np.asarray(rgp.gpytorch_predict2casadi(gps[i])(z=None)["mean"]).ravel()[0]))
        out[f"gp{i}_mean_q"] = np.array(means)
    _Eager.bind = {}

    # ---- a13: prior linearisation -> exact ZOH, DARE, LQR --------------------------
    Q, R = np.diag(spec.q_diag), np.diag(spec.r_diag)
    dfdx, dfdu = spec.prior_jacobian(np.zeros(12), spec.u_eq)
    Ad, Bd_u, K = rgpmpc.GPMPC.setup_prior_dynamics(dfdx, dfdu, Q, R, spec.dt)
    out["lqr_dfdx"], out["lqr_dfdu"], out["lqr_Ad"], out["lqr_Bd"], out["lqr_K"] = dfdx, dfdu, Ad, Bd_u, K

    # ---- a10: constraint tightening -------------------------------------------------
    T = 10
    x_prev = np.zeros((12, T + 1))
    x_prev[[0, 2]] = rng.uniform(-1, 1, (2, T + 1))
    x_prev[4] = 1.0 + 0.2 * rng.standard_normal(T + 1)
    x_prev[[1, 3, 5]] = 0.5 * rng.standard_normal((3, T + 1))
    x_prev[[6, 7, 8]] = 0.2 * rng.standard_normal((3, T + 1))
    x_prev[[9, 10, 11]] = 0.5 * rng.standard_normal((3, T + 1))
    u_prev = np.vstack([rng.uniform(0.15, 0.55, T), rng.uniform(-0.4, 0.4, (3, T))])
    prob = 0.95
    icdf = float(__import__("scipy").stats.norm.ppf(1 - (1 / 12 - (prob + 1) / (2 * 12))))
    me = types.SimpleNamespace(
        model=types.SimpleNamespace(nx=12, nu=4), T=T, x_prev=x_prev, u_prev=u_prev, device="cpu",
        gaussian_process=gps, gp_idx=gp_idx, dt=spec.dt, inverse_cdf=icdf, lqr_gain=K,
        discrete_dfdx=Ad, discrete_dfdu=Bd_u, Bd=np.eye(12)[:, [1, 3, 5, 9, 10]])
    sc, ic = rgpmpc.GPMPC.propagate_constraint_limits(me)
    out["tt_x_prev"], out["tt_u_prev"], out["tt_prob"], out["tt_icdf"] = x_prev, u_prev, prob, icdf
    out["tt_state"], out["tt_input"] = sc, ic
    me.x_prev = None
    sc0, ic0 = rgpmpc.GPMPC.propagate_constraint_limits(me)
    assert not sc0.any() and not ic0.any()

    # ---- a11: FITC precompute ----------------------------------------------------------
    M = 12
    me2 = types.SimpleNamespace(gaussian_process=gps, gp_idx=gp_idx, np_random=np.random.default_rng(1337))
    w, S = rgpmpc.GPMPC.precompute_sparse_posterior_mean(me2, M)
    out["fitc_M"], out["fitc_w"], out["fitc_S"] = M, w, S
    out["fitc_idx"] = np.random.default_rng(1337).choice(range(N), size=M, replace=False)

    # ---- a14 / a8: reference window, constraint rows ----------------------------------
    traj = spec.reference_trajectory(37)
    me3 = types.SimpleNamespace(traj=traj, traj_step=30, T=T)
    out["ref_traj"], out["ref_step"], out["ref_window"] = traj, 30, rgpmpc.GPMPC.reference_trajectory(me3)
    sym = rng.standard_normal(12)
    out["cstr_sym"] = sym
    out["cstr_rows"] = np.asarray(rgpmpc.GPMPC.setup_constraints(sym, spec.x_lo, spec.x_hi)).ravel()

    # ---- f(3): GPMPC.preprocess_data (training targets), prior supplied by the build's spec --
    n = 25
    px = np.zeros((n, 12))
    px[:, [0, 2, 4]] = rng.uniform(-1, 1, (n, 3))
    px[:, [1, 3, 5]] = 0.5 * rng.standard_normal((n, 3))
    px[:, 6:9] = 0.2 * rng.standard_normal((n, 3))
    px[:, 9:12] = 0.5 * rng.standard_normal((n, 3))
    pu = np.column_stack([rng.uniform(0.15, 0.55, n), rng.uniform(-0.4, 0.4, (n, 3))])
    pxn = px + 0.02 * rng.standard_normal((n, 12))

    class _Arr:
        def __init__(self, a):
            self.a = np.asarray(a)

        def full(self):
            return self.a

        def toarray(self):
            return self.a

    me4 = types.SimpleNamespace(
        acc_symbolic_fn=lambda T: _Arr(spec.prior["a"] * np.asarray(T) + spec.prior["b"]),
        prior_dynamics=lambda x, u: {"f": _Arr(spec.prior_f(x.T, u.T).T)})
    pin, pout = rgpmpc.GPMPC.preprocess_data(me4, px, pu, pxn)
    out["pp_x"], out["pp_u"], out["pp_xn"], out["pp_in"], out["pp_out"] = px, pu, pxn, pin, pout

    np.savez(HERE / "golden_quad3d.npz", **out)
    print("wrote", HERE / "golden_quad3d.npz", "keys:", len(out))


if __name__ == "__main__":
    main()
