"""Seeded synthetic workloads (SURVEY.md §8(d) "Synthetic inputs").

There is no network and no crazyflow simulator, so the training sets, initial states and
plant are synthetic:

* GP training inputs are uniform over an operating box of each GP's input dims.
* GP targets are the residual between the "true" plant parameters and the prior
  (``spec.true_params`` vs ``spec.prior``) in the rows the GP feeds, plus N(0, 1e-2^2)
  noise -- the quantity `gpmpc/gpmpc.py:113-151` (``preprocess_data``) estimates from
  transitions.
* Instance ``b`` starts at reference phase ``b mod L`` plus N(0, 0.05^2) per state.
"""

from __future__ import annotations

import numpy as np

from .models import MODEL_CARTPOLE, MODEL_QUAD2D, MODEL_QUAD3D, ModelSpec

# Operating boxes for the GP inputs, per input index of z = [x; u].
_QUAD_BOX = {"theta": (-0.6, 0.6), "dtheta": (-3.0, 3.0)}


def gp_input_box(spec: ModelSpec, gp: int) -> tuple[np.ndarray, np.ndarray]:
    lo, hi = [], []
    zlo = np.concatenate([spec.x_lo, spec.u_lo])
    zhi = np.concatenate([spec.x_hi, spec.u_hi])
    for j in spec.gp_inputs[gp]:
        a, b = zlo[j], zhi[j]
        if j < spec.nx:  # states: use the operating region, not the hard bounds
            if spec.model_id in (MODEL_QUAD2D, MODEL_QUAD3D):
                is_rate = (spec.model_id == MODEL_QUAD2D and j == 5) or (spec.model_id == MODEL_QUAD3D and j in (9, 10))
                a, b = _QUAD_BOX["dtheta"] if is_rate else _QUAD_BOX["theta"]
            else:
                a, b = (-0.5, 0.5) if j == 2 else (-2.0, 2.0)
        lo.append(a)
        hi.append(b)
    return np.array(lo), np.array(hi)


def _cartpole_acc(p: dict, g: float, th, w, F):
    mc, mp, l = p["m_c"], p["m_p"], p["l"]
    M = mc + mp
    s, c = np.sin(th), np.cos(th)
    tmp = (F + mp * l * w * w * s) / M
    tha = (g * s - c * tmp) / (l * (4.0 / 3.0 - mp * c * c / M))
    xa = tmp - mp * l * tha * c / M
    return xa, tha


def residual_targets(spec: ModelSpec, gp: int, Z: np.ndarray) -> np.ndarray:
    """Noise-free residual (true - prior) seen by GP ``gp`` at inputs Z (n, d)."""
    P, T = spec.prior, spec.true_params
    if spec.model_id in (MODEL_QUAD2D, MODEL_QUAD3D):
        name = spec.gp_names[gp]
        if name == "T":
            return (T["a"] - P["a"]) * Z[:, 0] + (T["b"] - P["b"])
        if name == "R":
            return (T["c"] - P["c"]) * Z[:, 0] + (T["d"] - P["d"]) * Z[:, 1] + (T["e"] - P["e"]) * Z[:, 2]
        if name == "P":
            return (T["f"] - P["f"]) * Z[:, 0] + (T["h"] - P["h"]) * Z[:, 1] + (T["l"] - P["l"]) * Z[:, 2]
    if spec.model_id == MODEL_CARTPOLE:
        xt, tt = _cartpole_acc(T, spec.gravity, Z[:, 0], Z[:, 1], Z[:, 2])
        xp, tp = _cartpole_acc(P, spec.gravity, Z[:, 0], Z[:, 1], Z[:, 2])
        return (xt - xp) if gp == 0 else (tt - tp)
    raise ValueError(spec.name)


def make_training_data(spec: ModelSpec, n: int, seed: int = 1, noise_std: float = 1e-2):
    """Per-GP training sets [(X (n,d), y (n,))] -- seeded (`gp_mpc_config.yaml:3`, seed 1)."""
    rng = np.random.default_rng(seed)
    out = []
    for g in range(spec.n_gp):
        lo, hi = gp_input_box(spec, g)
        X = rng.uniform(lo, hi, size=(n, len(lo)))
        y = residual_targets(spec, g, X) + noise_std * rng.standard_normal(n)
        out.append((X, y))
    return out


# Fixed hyperparameters for timing runs: (lengthscale, outputscale, noise).
DEFAULT_HYPERS = {
    "quad2d": [(0.2, 25.0, 1e-4), (2.0, 50.0, 1e-4)],
    "quad3d": [(0.2, 25.0, 1e-4), (2.0, 50.0, 1e-4), (2.0, 50.0, 1e-4)],
    # the scalar lengthscale spans [theta, dtheta, F] with F in [-10, 10]: 3 keeps the
    # residual mean smooth along F (1.0 made it ripple between the N=50 samples and the
    # Gauss-Newton SQP cycle)
    "cartpole": [(3.0, 4.0, 1e-4), (3.0, 16.0, 1e-4)],
}


def initial_states(spec: ModelSpec, traj: np.ndarray, batch: int, seed: int = 1, std: float = 0.05):
    """x0[b] = traj[:, b mod L] + N(0, std^2), phase[b] = b mod L."""
    rng = np.random.default_rng(seed + 1)
    L = traj.shape[1]
    phase = np.arange(batch) % L
    x0 = traj[:, phase].T + std * rng.standard_normal((batch, spec.nx))
    return x0, phase.astype(np.int32)
