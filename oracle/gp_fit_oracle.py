"""CPU oracle for the GP hyperparameter fit -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, and only as the checker; the product fit
(``gp-mpc_amd/gpmpc/gp.py`` ``exact_mll`` / ``fit_gp`` and ``gpmpc/distributed.py``
``mll_and_grad_partial`` / ``fit_gp_allreduce``) never imports it.

It restates in float64 numpy, independently of torch autograd, what the reference's fit does
(`gpmpc/gp.py:49-69`, called per GP by `gpmpc/gpmpc.py:153-164`):

* gpytorch's parameterisation of ``ScaleKernel(RBFKernel())`` + ``GaussianLikelihood``
  (`gpmpc/gp.py:31-34`): lengthscale = softplus(raw), outputscale = softplus(raw),
  noise = 1e-6 + softplus(raw) (``GreaterThan(1e-6)``); raw parameters start at 0.
* ``ExactMarginalLogLikelihood`` (`gpmpc/gp.py:57,62`): log N(y | 0, K + noise I) / n, with
  K = sf2 exp(-|x - x'|^2 / (2 ell^2)), evaluated by a Cholesky factorisation (gpytorch's path up
  to ``max_cholesky_size`` = 800 rows; above it gpytorch switches to CG / Lanczos estimates, which
  are stochastic and absent here: parity unpinned there).
* its analytic gradient with respect to the raw parameters,
  d(MLL/n)/d theta = tr((a a^T - K^-1) dK/dtheta) / (2n) times softplus'(raw) = sigmoid(raw),
  dK/d ell = sf2 E o D2 / ell^3, dK/d sf2 = E, dK/d noise = I (a = K^-1 y, E = exp(-D2 / 2ell^2)).
* ``torch.optim.Adam`` with its defaults (betas 0.9 / 0.999, eps 1e-8, no weight decay, no
  amsgrad), restated from its published update rule: m <- m + (1 - b1)(g - m),
  v <- b2 v + (1 - b2) g^2, p <- p - lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps).
* the reference's loop: ``n_train`` iterations of zero_grad / loss = -MLL / backward / step, then
  stop when |last_loss - loss| < 1e-3 (`gpmpc/gp.py:58-67`).

Pinning: gpytorch is not installed, so the MLL is pinned against its closed
form instead -- a 1-point GP by hand and scipy's multivariate normal log-density in
``tests/test_gp_fit_oracle.py`` -- and the gradient against central finite differences of the
MLL.  The Adam restatement is checked against torch.optim.Adam on a fixed gradient sequence.
"""

from __future__ import annotations

import math

import numpy as np

NOISE_LOWER = 1e-6   # GreaterThan(1e-6), gpmpc/gp.py:31


def softplus(x: float) -> float:
    return float(np.logaddexp(0.0, x))


def sigmoid(x: float) -> float:
    return float(1.0 / (1.0 + math.exp(-x)))


def constrained(raw: np.ndarray) -> tuple[float, float, float]:
    """(lengthscale, outputscale, noise) from the raw parameters (gpytorch constraints)."""
    return softplus(raw[0]), softplus(raw[1]), softplus(raw[2]) + NOISE_LOWER


def _sqdist(X: np.ndarray) -> np.ndarray:
    X = np.asarray(X, dtype=np.float64).reshape(X.shape[0], -1)
    return ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)


def mll(X: np.ndarray, y: np.ndarray, raw: np.ndarray) -> float:
    """Exact marginal log likelihood / n (ExactMarginalLogLikelihood, Cholesky path)."""
    y = np.asarray(y, dtype=np.float64)
    n = y.shape[0]
    ell, sf2, noise = constrained(raw)
    K = sf2 * np.exp(-0.5 * _sqdist(X) / ell**2) + noise * np.eye(n)
    L = np.linalg.cholesky(K)
    a = np.linalg.solve(L.T, np.linalg.solve(L, y))
    return float((-0.5 * y @ a - np.log(np.diag(L)).sum() - 0.5 * n * math.log(2 * math.pi)) / n)


def mll_grad(X: np.ndarray, y: np.ndarray, raw: np.ndarray) -> tuple[float, np.ndarray]:
    """MLL / n and its analytic gradient with respect to (raw lengthscale, raw outputscale, raw noise)."""
    y = np.asarray(y, dtype=np.float64)
    n = y.shape[0]
    ell, sf2, noise = constrained(raw)
    D2 = _sqdist(X)
    E = np.exp(-0.5 * D2 / ell**2)
    K = sf2 * E + noise * np.eye(n)
    L = np.linalg.cholesky(K)
    Linv = np.linalg.solve(L, np.eye(n))
    Kinv = Linv.T @ Linv
    a = Kinv @ y
    val = float((-0.5 * y @ a - np.log(np.diag(L)).sum() - 0.5 * n * math.log(2 * math.pi)) / n)
    W = np.outer(a, a) - Kinv
    g = np.array([
        (W * (sf2 * E * D2 / ell**3)).sum(),   # dK/d ell
        (W * E).sum(),                         # dK/d sf2
        np.trace(W),                           # dK/d noise = I
    ]) * (0.5 / n)
    chain = np.array([sigmoid(raw[0]), sigmoid(raw[1]), sigmoid(raw[2])])
    return val, g * chain


class Adam:
    """torch.optim.Adam(lr) with its default betas / eps, restated (see the module docstring)."""

    def __init__(self, lr: float, betas=(0.9, 0.999), eps: float = 1e-8):
        self.lr, (self.b1, self.b2), self.eps = float(lr), betas, float(eps)
        self.m = self.v = None
        self.t = 0

    def step(self, p: np.ndarray, grad: np.ndarray) -> np.ndarray:
        if self.m is None:
            self.m, self.v = np.zeros_like(p), np.zeros_like(p)
        self.t += 1
        self.m = self.m + (1.0 - self.b1) * (grad - self.m)
        self.v = self.b2 * self.v + (1.0 - self.b2) * grad * grad
        bc1 = 1.0 - self.b1**self.t
        bc2 = 1.0 - self.b2**self.t
        denom = np.sqrt(self.v) / math.sqrt(bc2) + self.eps
        return p - (self.lr / bc1) * self.m / denom


def fit(X: np.ndarray, y: np.ndarray, n_train: int = 500, lr: float = 0.01, raw0=None) -> dict:
    """The reference's ``fit_gp`` loop (`gpmpc/gp.py:58-67`) on the oracle's MLL gradient.

    Returns the raw parameters after every Adam step (``raw``, (iters, 3)), the loss evaluated
    before each step (``loss``), the number of steps taken and, for tests, the smallest distance of
    an early-stop comparison to its 1e-3 threshold (``stop_margin``)."""
    raw = np.zeros(3) if raw0 is None else np.asarray(raw0, dtype=np.float64).copy()
    opt = Adam(lr)
    last = math.inf
    hist_raw, hist_loss, margin = [], [], math.inf
    for _ in range(n_train):
        val, g = mll_grad(X, y, raw)
        loss = -val
        raw = opt.step(raw, -g)            # gradient of the loss = -MLL
        hist_raw.append(raw.copy())
        hist_loss.append(loss)
        if math.isfinite(last):
            margin = min(margin, abs(abs(last - loss) - 1e-3))
        if abs(last - loss) < 1e-3:
            break
        last = loss
    return {"raw": np.array(hist_raw), "loss": np.array(hist_loss), "iters": len(hist_loss), "stop_margin": margin}
