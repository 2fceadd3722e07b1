"""Numpy model of the segment-parallel Newton solve (gp-mpc_amd/csrc/sqp_kernel.hip, SqpKernel
kSeg: seg_factor / seg_chain_full / seg_chain_vec / seg_fold / seg_forward) against the dense KKT
solve of the IPM's Newton system (CPU, no GPU).

The system is the LQ problem over stages 0..H with dx_0 = 0 (the Riccati recursion's own problem,
reference: acados/HPIPM's Riccati solve inside `gpmpc/gpmpc.py:364`'s `solver.solve()`):
    min sum_k 1/2 w_k' diag(h_k) w_k + g_k' w_k,   x_{k+1} = A_k x_k + B_k u_k + c_k.
The horizon splits into segments at floor(s H / NSEG); every segment but the last runs the Riccati
recursion over z = [x; 1; lam] from the terminal cost lam' x_b (lam: the unknown costate of its end
state), the last one from the true terminal cost.  The boundary chain solves for the costates
backwards with T_b^-1 = Ph M^-1, M = Ph + Ph W Ph (W = -V_ll), then runs forward over the
boundaries; every segment then sweeps forward on its own.  The corrector reuses T_b^-1, Y_b and
the chained cost-to-go matrices with new vectors only.
"""

import numpy as np
import pytest


def _problem(rng, H, nx, nu):
    A = [np.eye(nx) + 0.1 * rng.standard_normal((nx, nx)) for _ in range(H)]
    B = [0.3 * rng.standard_normal((nx, nu)) for _ in range(H)]
    c = [0.05 * rng.standard_normal(nx) for _ in range(H)]
    h = [np.concatenate([rng.uniform(0.5, 3.0, nx), rng.uniform(0.1, 1.0, nu)]) for _ in range(H + 1)]
    g = [0.2 * rng.standard_normal(nx + nu) for _ in range(H + 1)]
    return A, B, c, h, g


def _kkt(A, B, c, h, g, H, nx, nu):
    """Dense KKT solve: primal w_k = [x_k; u_k] (u_H unused) with x_0 = 0."""
    nb = nx + nu
    nv, ne = (H + 1) * nb, (H + 1) * nx
    K = np.zeros((nv + ne, nv + ne))
    rhs = np.zeros(nv + ne)
    for k in range(H + 1):
        K[k * nb:(k + 1) * nb, k * nb:(k + 1) * nb] = np.diag(h[k])
        rhs[k * nb:(k + 1) * nb] = -g[k]
    for i in range(nx):
        K[nv + i, i] = K[i, nv + i] = 1.0
    for k in range(H):
        r0 = nv + (k + 1) * nx
        rows = np.zeros((nx, nv))
        rows[:, (k + 1) * nb:(k + 1) * nb + nx] = np.eye(nx)
        rows[:, k * nb:k * nb + nx] = -A[k]
        rows[:, k * nb + nx:(k + 1) * nb] = -B[k]
        K[r0:r0 + nx, :nv] = rows
        K[:nv, r0:r0 + nx] = rows.T
        rhs[r0:r0 + nx] = c[k]
    w = np.linalg.solve(K, rhs)[:nv].reshape(H + 1, nb)
    return w[:, :nx], w[:H, nx:]


def _gauss_jordan_spd(M, R):
    """Gauss-Jordan without pivoting on [M | R] (M symmetric positive definite): M^-1 R."""
    a = np.concatenate([M, R], axis=1).copy()
    n = M.shape[0]
    for p in range(n):
        a[p] /= a[p, p]
        for i in range(n):
            if i != p:
                a[i] -= a[i, p] * a[p]
    return a[:, n:]


def _segment_factor(A, B, c, h, g, k0, k1, nx, nu, Pterm):
    """Riccati over z = [x; 1; lam] (lam of dimension nx; last segment: lam unused, Pterm the true
    terminal cost in z coordinates).  Returns the z-space cost-to-go P_k0 and the feedbacks K_k
    (u_k = K_k z_k)."""
    nz = 2 * nx + 1
    CI = nx
    P = Pterm
    Ks = {}
    for k in range(k1 - 1, k0 - 1, -1):
        Az = np.eye(nz)
        Az[:nx, :nx] = A[k]
        Az[:nx, CI] = c[k]
        Bz = np.zeros((nz, nu))
        Bz[:nx] = B[k]
        Qz = np.zeros((nz, nz))
        Qz[:nx, :nx] = np.diag(h[k][:nx])
        Qz[:nx, CI] = Qz[CI, :nx] = g[k][:nx]
        Quu = np.diag(h[k][nx:]) + Bz.T @ P @ Bz
        Qux = Bz.T @ P @ Az
        Qux[:, CI] += g[k][nx:]
        Kk = -np.linalg.solve(Quu, Qux)
        P = Qz + Az.T @ P @ Az + Qux.T @ Kk
        P = 0.5 * (P + P.T)
        Ks[k] = Kk
    return P, Ks


def _terminal(h, g, H, nx, lam):
    nz = 2 * nx + 1
    P = np.zeros((nz, nz))
    if lam:   # lam' x_b
        P[:nx, nx + 1:] = np.eye(nx)
        P[nx + 1:, :nx] = np.eye(nx)
    else:     # the true terminal stage cost
        P[:nx, :nx] = np.diag(h[H][:nx])
        P[:nx, nx] = P[nx, :nx] = g[H][:nx]
    return P


def _segment_solve(A, B, c, h, g, H, nx, nu, nseg, chain=None):
    """The kernel's algorithm; chain = the predictor's stored (T^-1, Y, Ph) for a corrector pass."""
    CI, L = nx, slice(nx + 1, 2 * nx + 1)
    starts = [(s * H) // nseg for s in range(nseg + 1)]
    seg = [_segment_factor(A, B, c, h, g, starts[s], starts[s + 1], nx, nu,
                           _terminal(h, g, H, nx, s < nseg - 1)) for s in range(nseg)]
    # cost-to-go at the last segment's start: its z-space P restricted to [x; 1]
    Plast = seg[-1][0]
    Ph, ph = Plast[:nx, :nx], Plast[:nx, CI]
    stored = {}
    y = {}
    Y = {}
    for b in range(nseg - 2, -1, -1):
        V = seg[b][0]
        Vll, Vlx, Vl1 = V[L, L], V[L, :nx], V[L, CI]
        if chain is None:
            W = -Vll
            assert np.linalg.eigvalsh(W).min() > -1e-9   # the segment's value is concave in lam
            M = Ph + Ph @ W @ Ph
            R = np.concatenate([Ph @ Vlx, (Ph @ Vl1 + ph)[:, None], np.eye(nx)], axis=1)
            out = Ph @ _gauss_jordan_spd(M, R)
            Y[b], y[b], Ti = out[:, :nx], out[:, nx], out[:, nx + 1:]
            np.testing.assert_allclose(Ti, np.linalg.inv(np.eye(nx) - Ph @ Vll), rtol=1e-10, atol=1e-12)
            stored[b] = (Ti, Y[b], Ph)
        else:   # corrector: factorisation unchanged, vectors only
            Ti, Y[b], Phs = chain[b]
            y[b] = Ti @ (Phs @ Vl1 + ph)
            Ph = Phs
        # cost-to-go at the segment's start for the next boundary
        Ph, ph = V[:nx, :nx] + V[:nx, L] @ Y[b], V[:nx, CI] + V[:nx, L] @ y[b]
        Ph = 0.5 * (Ph + Ph.T)
    # forward over the boundaries, then every segment's sweep
    xs = np.zeros((H + 1, nx))
    us = np.zeros((H, nu))
    xb = np.zeros(nx)
    for s in range(nseg):
        lam = (Y[s] @ xb + y[s]) if s < nseg - 1 else np.zeros(nx)
        x = xb
        for k in range(starts[s], starts[s + 1]):
            z = np.concatenate([x, [1.0], lam])
            u = seg[s][1][k] @ z
            xs[k], us[k] = x, u
            x = A[k] @ x + B[k] @ u + c[k]
        xb = x
    xs[H] = xb
    return xs, us, stored


@pytest.mark.parametrize("H,nseg", [(10, 3), (10, 2), (4, 3), (7, 3), (30, 3), (30, 2)])
@pytest.mark.parametrize("nx,nu", [(6, 2), (4, 1)])
def test_segment_solve_matches_dense_kkt(H, nseg, nx, nu):
    rng = np.random.default_rng(1000 * H + 10 * nx + nseg)
    A, B, c, h, g = _problem(rng, H, nx, nu)
    xk, uk = _kkt(A, B, c, h, g, H, nx, nu)
    xs, us, stored = _segment_solve(A, B, c, h, g, H, nx, nu, nseg)
    np.testing.assert_allclose(xs, xk, rtol=0, atol=1e-9 * (1 + np.abs(xk).max()))
    np.testing.assert_allclose(us, uk, rtol=0, atol=1e-9 * (1 + np.abs(uk).max()))
    # corrector: new gradient and dynamics residual, the chain's matrices reused
    g2 = [gi + 0.1 * rng.standard_normal(gi.shape) for gi in g]
    c2 = [ci + 0.01 * rng.standard_normal(ci.shape) for ci in c]
    xk2, uk2 = _kkt(A, B, c2, h, g2, H, nx, nu)
    xs2, us2, _ = _segment_solve(A, B, c2, h, g2, H, nx, nu, nseg, chain=stored)
    np.testing.assert_allclose(xs2, xk2, rtol=0, atol=1e-9 * (1 + np.abs(xk2).max()))
    np.testing.assert_allclose(us2, uk2, rtol=0, atol=1e-9 * (1 + np.abs(uk2).max()))


def test_spd_form_of_the_boundary_inverse():
    """T = I - Ph V_ll with Ph > 0 and V_ll <= 0: T^-1 = Ph (Ph + Ph W Ph)^-1, W = -V_ll, and the
    pivot-free Gauss-Jordan elimination on that symmetric positive-definite matrix is accurate even
    where T itself has a vanishing leading minor (which pivot-free elimination on T would divide by)."""
    rng = np.random.default_rng(7)
    for _ in range(50):
        n = 6
        Q = rng.standard_normal((n, n))
        Ph = Q @ Q.T + 0.1 * np.eye(n)
        Z = rng.standard_normal((n, 3))
        W = Z @ Z.T
        T = np.eye(n) + Ph @ W
        M = Ph + Ph @ W @ Ph
        Ti = Ph @ _gauss_jordan_spd(M, np.eye(n))
        np.testing.assert_allclose(Ti @ T, np.eye(n), atol=1e-8)
    # a T with T[0, 0] = 0: Ph = [[1, -3], [-3, 10]] > 0, W = [[2, 1], [1, 1]] >= 0, (Ph W)[0, 0] = -1
    Ph = np.array([[1.0, -3.0], [-3.0, 10.0]])
    W = np.array([[2.0, 1.0], [1.0, 1.0]])
    T = np.eye(2) + Ph @ W
    assert abs(T[0, 0]) < 1e-12
    Ti = Ph @ _gauss_jordan_spd(Ph + Ph @ W @ Ph, np.eye(2))
    np.testing.assert_allclose(Ti @ T, np.eye(2), atol=1e-12)
