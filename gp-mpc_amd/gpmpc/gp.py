"""Gaussian processes for the GP-MPC solve path (drop-in for ``gpmpc/gp.py``).

* :class:`GaussianProcess` -- exact GP, zero mean, isotropic SE kernel (``ScaleKernel(RBFKernel())``),
  Gaussian likelihood with noise >= 1e-6 (`gpmpc/gp.py:24-46`).  ``predict()`` is the build's
  GP posterior surface: mean and exact variance on the MI355X through the C ABI
  (``gpmpc_gp_posterior``), no CPU fallback.
* :func:`fit_gp` -- Adam on the exact negative marginal log likelihood with early stopping
  (`gpmpc/gp.py:49-69`).  Host-side torch autograd with a Cholesky MLL; it runs once per
  learning epoch, off the control-step hot path.
* :func:`covSE_single` / :func:`covSE_vectorized` -- the SE kernel (`gpmpc/gp.py:12-21`) on
  numpy/torch arrays (CasADi is not part of this build).
"""

from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib

NOISE_LOWER = 1e-6  # GreaterThan(1e-6), gpmpc/gp.py:31


def covSE_single(x, z, ell, sf2):
    """sf2 * exp(-0.5 * sum_rows((x - z)^2 / ell^2)) with x, z column-stacked (d, n)."""
    mod = torch if isinstance(x, torch.Tensor) else np
    dist = ((x - z) ** 2 / ell**2).sum(0)
    return sf2 * mod.exp(-0.5 * dist)


def covSE_vectorized(x, Z, ell, sf2):
    """Kernel between one point x (d,) or (d,1) and the rows of Z (M, d)."""
    x = x.reshape(-1, 1)
    return covSE_single(x, Z.T, ell, sf2)


def _softplus_inv(v: float) -> float:
    return v + math.log(-math.expm1(-v))


class GaussianProcess:
    """Exact GP with zero mean and an isotropic SE kernel (`gpmpc/gp.py:24-46`).

    Hyperparameters are stored as softplus-constrained raw parameters like gpytorch
    (lengthscale, outputscale, noise = 1e-6 + softplus(raw)), so :func:`fit_gp` optimises the
    same parameterisation.
    """

    def __init__(self, x: torch.Tensor, y: torch.Tensor, lengthscale: float = math.log(2.0),
                 outputscale: float = math.log(2.0), noise: float = math.log(2.0) + NOISE_LOWER):
        assert isinstance(x, torch.Tensor), "x must be a torch.Tensor"
        assert isinstance(y, torch.Tensor), "y must be a torch.Tensor"
        x = x.to(torch.float64)
        if x.ndim == 1:
            x = x[:, None]
        self.train_inputs = (x,)
        self.train_targets = y.to(torch.float64).reshape(-1)
        if self.train_targets.shape[0] != x.shape[0]:
            raise ValueError("x and y disagree on the number of points")
        if not 1 <= x.shape[1] <= 3:
            raise ValueError("the MI355X kernels take GP input dimension 1..3")
        self.n_ind_points = x.shape[0]
        self.input_dimension = x.shape[1]
        dev, dt = x.device, torch.float64
        self.raw_lengthscale = torch.tensor(_softplus_inv(lengthscale), device=dev, dtype=dt)
        self.raw_outputscale = torch.tensor(_softplus_inv(outputscale), device=dev, dtype=dt)
        self.raw_noise = torch.tensor(_softplus_inv(max(noise - NOISE_LOWER, 1e-12)), device=dev, dtype=dt)
        self.K, self.K_inv = None, None  # only computed once the GP is trained
        self._dev = None

    # ---------------------------------------------------------------- hyperparameters
    @property
    def lengthscale(self) -> float:
        return float(torch.nn.functional.softplus(self.raw_lengthscale))

    @property
    def outputscale(self) -> float:
        return float(torch.nn.functional.softplus(self.raw_outputscale))

    @property
    def noise(self) -> float:
        return float(torch.nn.functional.softplus(self.raw_noise)) + NOISE_LOWER

    def set_hyperparameters(self, lengthscale: float, outputscale: float, noise: float):
        self.raw_lengthscale.fill_(_softplus_inv(lengthscale))
        self.raw_outputscale.fill_(_softplus_inv(outputscale))
        self.raw_noise.fill_(_softplus_inv(max(noise - NOISE_LOWER, 1e-12)))
        self.K, self.K_inv, self._dev = None, None, None
        return self

    def parameters(self):
        return [self.raw_lengthscale, self.raw_outputscale, self.raw_noise]

    def to(self, device):
        self.train_inputs = (self.train_inputs[0].to(device),)
        self.train_targets = self.train_targets.to(device)
        for name in ("raw_lengthscale", "raw_outputscale", "raw_noise"):
            setattr(self, name, getattr(self, name).detach().to(device))
        self.K, self.K_inv, self._dev = None, None, None
        return self

    # ---------------------------------------------------------------- covariances
    def kernel(self, a: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
        b = a if b is None else b
        ell = torch.nn.functional.softplus(self.raw_lengthscale)
        sf2 = torch.nn.functional.softplus(self.raw_outputscale)
        d2 = torch.cdist(a, b).pow(2) if a.shape[1] > 1 else (a - b.T).pow(2)
        return sf2 * torch.exp(-0.5 * d2 / ell**2)

    def compute_covariances(self) -> tuple[torch.Tensor, torch.Tensor]:
        """K = k(X,X) + noise*I and its inverse (`gpmpc/gp.py:43-46`)."""
        with torch.no_grad():
            X = self.train_inputs[0]
            K = self.kernel(X) + self.noise * torch.eye(X.shape[0], dtype=X.dtype, device=X.device)
            return K, torch.linalg.inv(K)

    def device_layout(self, device=None) -> dict:
        """GP data in the kernel layout: rows [npad][4] = (x, alpha), linvT = (L^-1)^T, padded."""
        if self._dev is not None and (device is None or self._dev["rows"].device == torch.device(device)):
            return self._dev
        if self.K is None:
            self.K, self.K_inv = self.compute_covariances()
        dev = torch.device(device) if device is not None else self.train_inputs[0].device
        X = self.train_inputs[0].to(dev)
        K = self.K.to(dev)
        y = self.train_targets.to(dev)
        alpha = self.K_inv.to(dev) @ y  # the reference's weights K_inv @ y (gpmpc/gp.py:84-85)
        L = torch.linalg.cholesky(K)
        eye = torch.eye(K.shape[0], dtype=K.dtype, device=dev)
        Linv = torch.linalg.solve_triangular(L, eye, upper=False)
        n, d = X.shape
        npad = (n + 15) // 16 * 16
        rows = torch.zeros(npad, 4, dtype=torch.float64, device=dev)
        rows[:n, :d] = X
        rows[:n, 3] = alpha
        linvT = torch.zeros(npad, npad, dtype=torch.float64, device=dev)
        linvT[:n, :n] = torch.tril(Linv).T
        self._dev = dict(rows=rows.contiguous(), linvT=linvT.contiguous(), n=n, d=d, npad=npad, alpha=alpha,
                         Linv=torch.tril(Linv))
        return self._dev

    # ---------------------------------------------------------------- LOVE root
    @torch.no_grad()
    def love_root(self, rank: int = 100, seed: int = 0) -> torch.Tensor:
        """Rank-r root R (n, r) with R R^T ~ (K + noise I)^-1: the predictive-covariance cache
        gpytorch builds under ``fast_pred_var`` (LOVE), which the reference's tightening uses
        (`gpmpc/gpmpc.py:442-444`).  Restated from gpytorch / linear_operator
        (``root_inv_decomposition`` -> ``lanczos_tridiag``, full reorthogonalisation;
        ``max_root_decomposition_size`` = 100 by default): Lanczos on K + noise I from a normal
        start vector, T = V diag(lam) V^T, R = Q V diag(lam)^-1/2.  gpytorch draws the start
        vector from torch's global generator; here it is seeded (``seed``).  gpytorch takes this
        path only above ``max_cholesky_size`` (800 rows) and the exact Cholesky root below it
        (see ``love_rows``)."""
        if self.K is None:
            self.K, self.K_inv = self.compute_covariances()
        K = self.K
        n = K.shape[0]
        k = min(int(rank), n)
        gen = torch.Generator(device="cpu").manual_seed(int(seed))
        q = torch.randn(n, dtype=torch.float64, generator=gen).to(K.device)
        Q = torch.zeros(n, k, dtype=torch.float64, device=K.device)
        alpha = torch.zeros(k, dtype=torch.float64, device=K.device)
        beta = torch.zeros(k, dtype=torch.float64, device=K.device)
        q = q / q.norm()
        m = k
        for j in range(k):
            Q[:, j] = q
            v = K @ q
            alpha[j] = q @ v
            v = v - alpha[j] * q - (beta[j - 1] * Q[:, j - 1] if j > 0 else 0.0)
            for _ in range(2):   # full reorthogonalisation (twice is enough)
                v = v - Q[:, : j + 1] @ (Q[:, : j + 1].T @ v)
            b = v.norm()
            if j + 1 == k or b <= 1e-12 * alpha[: j + 1].abs().max():
                m = j + 1
                break
            beta[j] = b
            q = v / b
        T = torch.diag(alpha[:m]) + torch.diag(beta[: m - 1], 1) + torch.diag(beta[: m - 1], -1)
        lam, V = torch.linalg.eigh(T)
        lam = lam.clamp_min(torch.finfo(torch.float64).tiny)
        return (Q[:, :m] @ V) * lam.rsqrt()

    # ---------------------------------------------------------------- posterior on the GPU
    @torch.no_grad()
    def predict(self, z: torch.Tensor, with_noise: bool = False, return_var: bool = True):
        """Posterior mean and exact variance at z (P, d) on the MI355X.

        ``with_noise`` adds the likelihood noise like ``gp.likelihood(gp(z))``
        (`gpmpc/gpmpc.py:444`).  Returns (mean, var) float64 tensors on z's device
        (var is None if ``return_var`` is False).
        """
        lib = _lib.load()
        if z.device.type != "cuda":
            raise _lib.GPMPCError("GaussianProcess.predict runs on the GPU: pass a cuda tensor")
        z = z.to(torch.float64)
        if z.ndim == 1:
            z = z[:, None] if self.input_dimension == 1 else z[None, :]
        z = z.contiguous()
        if z.shape[1] != self.input_dimension:
            raise ValueError(f"expected points of dimension {self.input_dimension}, got {z.shape[1]}")
        lay = self.device_layout(z.device)
        P = z.shape[0]
        mean = torch.empty(P, dtype=torch.float64, device=z.device)
        var = torch.empty(P, dtype=torch.float64, device=z.device) if return_var else None
        _lib.check(lib.gpmpc_gp_posterior(
            lay["n"], lay["d"], lay["npad"], _lib.ptr(lay["rows"]), _lib.ptr(lay["linvT"]) if return_var else None,
            self.lengthscale, self.outputscale, self.noise, _lib.ptr(z), P, _lib.ptr(mean), _lib.ptr(var),
            int(with_noise), _lib.stream_ptr(z.device)))
        return mean, var


def exact_mll(gp: GaussianProcess) -> torch.Tensor:
    """Exact marginal log likelihood / N (gpytorch ExactMarginalLogLikelihood convention)."""
    X, y = gp.train_inputs[0], gp.train_targets
    n = X.shape[0]
    noise = torch.nn.functional.softplus(gp.raw_noise) + NOISE_LOWER
    K = gp.kernel(X) + noise * torch.eye(n, dtype=X.dtype, device=X.device)
    L = torch.linalg.cholesky(K)
    a = torch.cholesky_solve(y[:, None], L)[:, 0]
    ll = -0.5 * (y @ a) - torch.log(torch.diagonal(L)).sum() - 0.5 * n * math.log(2 * math.pi)
    return ll / n


def fit_gp(gp: GaussianProcess, n_train: int = 500, lr: float = 0.01, device: str = "cpu",
           history: list | None = None) -> int:
    """Adam on -MLL with early stopping |dloss| < 1e-3, then K, K_inv (`gpmpc/gp.py:49-69`).

    Returns the number of Adam steps taken.  ``history`` (optional list) receives one
    ``(loss before the step, raw parameters after it)`` pair per step, for the parity tests
    against the fit oracle (oracle/gp_fit_oracle.py)."""
    assert isinstance(gp, GaussianProcess), f"gp must be a GaussianProcess, got {type(gp)}"
    gp.to(device)
    params = gp.parameters()
    for p in params:
        p.requires_grad_(True)
    optim = torch.optim.Adam(params, lr=lr)
    last = math.inf
    it = 0
    for it in range(1, n_train + 1):
        optim.zero_grad()
        loss = -exact_mll(gp)
        loss.backward()
        optim.step()
        lv = float(loss.detach())
        if history is not None:
            history.append((lv, [float(p.detach()) for p in params]))
        if abs(last - lv) < 1e-3:
            break
        last = lv
    for p in params:
        p.requires_grad_(False)
    gp._dev = None
    gp.K, gp.K_inv = gp.compute_covariances()
    return it


# gpytorch.settings.max_cholesky_size default: below it the LOVE cache is the exact Cholesky root
LOVE_CHOLESKY_ROWS = 800
