"""Prototype (diagnostic only): the IPM Newton system of the oracle's QP solved through the dual
Schur complement Y = C H^-1 C^T (block tridiagonal, T blocks of nx) by odd-even cyclic reduction,
against the dense KKT solve.  Runs oracle closed loops with both linear solvers and compares the
IPM iteration counts and the trajectories.

    python tools/cr_proto.py [--model quad2d] [--n-train 200] [--horizon 30] [--batch 4] [--steps 12]
"""

from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gp-mpc_amd"), str(ROOT), str(ROOT / "tests")]

from helpers import O, initial_states, lqr, oracle_gps, oracle_step, problem  # noqa: E402


def cr_solve(D, E, r, stats=None):
    """Block tridiagonal SPD solve: D[k] = Y[k,k], E[k] = Y[k+1,k], rhs r[k]; odd-even cyclic reduction."""
    n = len(D)
    if n == 1:
        return [np.linalg.solve(D[0], r[0])]
    Di = {i: np.linalg.inv(D[i]) for i in range(1, n, 2)}
    ev = list(range(0, n, 2))
    D2, E2, r2 = [], [], []
    for j in ev:
        d = D[j].copy()
        rr = r[j].copy()
        if j - 1 >= 0:
            d -= E[j - 1] @ Di[j - 1] @ E[j - 1].T
            rr -= E[j - 1] @ Di[j - 1] @ r[j - 1]
        if j + 1 < n:
            d -= E[j].T @ Di[j + 1] @ E[j]
            rr -= E[j].T @ Di[j + 1] @ r[j + 1]
        D2.append(d)
        r2.append(rr)
        if j + 2 < n:
            E2.append(-E[j + 1] @ Di[j + 1] @ E[j])
    y2 = cr_solve(D2, E2, r2, stats)
    y = [None] * n
    for q, j in enumerate(ev):
        y[j] = y2[q]
    for i in range(1, n, 2):
        rr = r[i] - E[i - 1] @ y[i - 1]
        if i + 1 < n:
            rr = rr - E[i].T @ y[i + 1]
        y[i] = Di[i] @ rr
    return y


class CRQP(O.DenseQP):
    """DenseQP whose Newton systems go through the dual Schur complement + cyclic reduction."""

    log: list = []

    def solve(self, lb, ub, tol=1e-10, max_iter=100, mu0=1.0):
        nx, T = self.nx, self.T
        C = self.C
        orig = np.linalg.solve

        def kkt_solve(K, rhs):
            n = self.n
            if K.shape[0] != n + self.m:
                return orig(K, rhs)
            h = np.diag(K[:n, :n])
            f, g = rhs[:n], rhs[n:]          # H dd + C^T dp = f, C dd = g
            hi = 1.0 / h
            Y = (C * hi) @ C.T
            rr = C @ (hi * f) - g
            D = [Y[k * nx:(k + 1) * nx, k * nx:(k + 1) * nx] for k in range(T)]
            E = [Y[(k + 1) * nx:(k + 2) * nx, k * nx:(k + 1) * nx] for k in range(T - 1)]
            dp = np.concatenate(cr_solve(D, E, [rr[k * nx:(k + 1) * nx] for k in range(T)]))
            dd = hi * (f - C.T @ dp)
            ref = orig(K, rhs)
            err = np.abs(np.concatenate([dd, dp]) - ref).max() / (1.0 + np.abs(ref).max())
            CRQP.log.append((err, h.max() / h.min()))
            return np.concatenate([dd, dp])

        np.linalg.solve = kkt_solve
        try:
            return super().solve(lb, ub, tol=tol, max_iter=max_iter, mu0=mu0)
        finally:
            np.linalg.solve = orig


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="quad2d")
    ap.add_argument("--n-train", type=int, default=200)
    ap.add_argument("--horizon", type=int, default=30)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--steps", type=int, default=12)
    a = ap.parse_args()
    spec, data, hyp = problem(a.model, a.n_train)
    gpo = oracle_gps(data, hyp)
    mats = lqr(spec)
    sd = spec.to_dict()
    H, B = a.horizon, a.batch
    opts = O.SQPOptions()
    traj = spec.reference_trajectory()
    plant = O.Dynamics(sd, None, params=spec.true_params)
    runs = {}
    for mode in ("dense", "cr"):
        sols = [O.SQPSolver(sd, O.Dynamics(sd, gpo), H, opts) for _ in range(B)]
        if mode == "cr":
            for s in sols:
                s.qp.__class__ = CRQP
        x0, phase = initial_states(spec, traj, B)
        prev = [None] * B
        hist = []
        for step in range(a.steps):
            for b in range(B):
                st, _, _ = oracle_step(spec, sols[b], gpo, x0[b], int(phase[b]) + step, H, traj, prev[b], lqr_mats=mats)
                hist.append((step, b, st, sols[b].sqp_iter, sum(sols[b].qp_iters), sols[b].x.copy(), sols[b].u.copy()))
                prev[b] = (sols[b].x.T.copy(), sols[b].u.T.copy())
                x0[b] = plant.rk4(x0[b], sols[b].u[0])[0]
        runs[mode] = hist
    worst = 0.0
    for hd, hc in zip(runs["dense"], runs["cr"]):
        ex = np.abs(hd[5] - hc[5]).max() / (1 + np.abs(hd[5]).max())
        eu = np.abs(hd[6] - hc[6]).max() / (1 + np.abs(hd[6]).max())
        worst = max(worst, ex, eu)
        if hd[2:5] != hc[2:5]:
            print(f"step {hd[0]} inst {hd[1]}: dense status/sqp/qp {hd[2:5]}  cr {hc[2:5]}")
    it_d = sum(h[4] for h in runs["dense"])
    it_c = sum(h[4] for h in runs["cr"])
    errs = np.array([e for e, _ in CRQP.log])
    conds = np.array([c for _, c in CRQP.log])
    print(f"IPM iterations dense {it_d}  cr {it_c};  trajectories max rel diff {worst:.3e}")
    print(f"CR vs dense Newton step: median {np.median(errs):.2e}  max {errs.max():.2e}  (diag H ratio up to {conds.max():.1e})")


if __name__ == "__main__":
    main()
