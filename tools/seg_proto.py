#!/usr/bin/env python3
"""Numpy prototype of the segment-parallel Newton solve of sqp_kernel.hip (kSeg).

The IPM's Newton system is an LQ problem over stages 0..H with dx_0 = 0:
    min sum_k 1/2 w_k^T diag(h_k) w_k + g_k^T w_k,  dx_{k+1} = A_k dx_k + B_k du_k + c_k.
Reference: the dense KKT solve.  Segment method: each of four segments runs the Riccati
recursion over z = [x; 1; lambda] with terminal cost lambda^T x_b (the last segment: the true
terminal cost), then the boundary chain solves for lambda_w (seg_boundary), then each segment
sweeps forward from x^_w with u = K x + kff + K_lambda lambda.  Also checks the corrector form
(factor fixed, new gradient g): p recursion with p_b = 0 plus V_l1 = sum P_lx,k+1 (c + B kff).

    python tools/seg_proto.py
"""

import numpy as np


def kkt_solve(A, B, c, h, g, H, nx, nu):
    nb = nx + nu
    nv = (H + 1) * nb
    ne = (H + 1) * nx   # dx_0 = 0 and H dynamics rows
    K = np.zeros((nv + ne, nv + ne))
    rhs = np.zeros(nv + ne)
    for k in range(H + 1):
        K[k * nb:(k + 1) * nb, k * nb:(k + 1) * nb] = np.diag(h[k])
        rhs[k * nb:(k + 1) * nb] = -g[k]
    # dx_0 = 0
    for i in range(nx):
        K[nv + i, i] = 1.0
        K[i, nv + i] = 1.0
    for k in range(H):
        r0 = nv + (k + 1) * nx
        for i in range(nx):
            K[r0 + i, (k + 1) * nb + i] = 1.0
            K[r0 + i, k * nb:k * nb + nx] = -A[k][i]
            K[r0 + i, k * nb + nx:k * nb + nb] = -B[k][i]
            rhs[r0 + i] = c[k][i]
        K[k * nb:(k + 1) * nb, r0:r0 + nx] = K[r0:r0 + nx, k * nb:(k + 1) * nb].T
        K[(k + 1) * nb:(k + 1) * nb + nx, r0:r0 + nx] = np.eye(nx)
    sol = np.linalg.solve(K, rhs)
    return sol[:nv].reshape(H + 1, nb)


def seg_factor(A, B, c, h, g, a0, b0, last, nx, nu, H):
    """Riccati over z = [x; 1; lam] for stages a0..b0-1.  Returns per-stage K' = [K | kff | K_l],
    P' blocks (full (2nx+1)^2) for stages a0..b0 (b0: terminal)."""
    nz = 2 * nx + 1
    P = np.zeros((nz, nz))
    if last:
        P[:nx, :nx] = np.diag(h[H][:nx])
        P[:nx, nx] = g[H][:nx]
        P[nx, :nx] = g[H][:nx]
    else:
        P[:nx, nx + 1:] = np.eye(nx)
        P[nx + 1:, :nx] = np.eye(nx)
    Ps = {b0: P.copy()}
    Ks, Rui = {}, {}
    for k in range(b0 - 1, a0 - 1, -1):
        # G'' maps [x; 1; lam; u] -> [x'; 1; lam']
        G = np.zeros((nz, nz + nu))
        G[:nx, :nx] = A[k]
        G[:nx, nx] = c[k]
        G[:nx, nz:] = B[k]
        G[nx, nx] = 1.0
        G[nx + 1:, nx + 1:nz] = np.eye(nx)
        D = np.zeros((nz + nu, nz + nu))
        D[:nx, :nx] = np.diag(h[k][:nx])
        D[nz:, nz:] = np.diag(h[k][nx:])
        D[:nx, nx] = D[nx, :nx] = g[k][:nx]
        D[nz:, nx] = D[nx, nz:] = g[k][nx:]
        M = G.T @ P @ G + D
        Ru = M[nz:, nz:]
        Ri = np.linalg.inv(Ru)
        Kp = -Ri @ M[nz:, :nz]
        P = M[:nz, :nz] + M[:nz, nz:] @ Kp
        Ps[k], Ks[k], Rui[k] = P.copy(), Kp, Ri
    return Ps, Ks, Rui


def seg_solve(A, B, c, h, g, H, nx, nu, nseg=4):
    st = [(w * H) // nseg for w in range(nseg + 1)]
    segs = [seg_factor(A, B, c, h, g, st[w], st[w + 1], w == nseg - 1, nx, nu, H) for w in range(nseg)]
    L = nx + 1
    # boundary chain
    P3 = segs[-1][0][st[nseg - 1]]
    Ph, ph = P3[:nx, :nx].copy(), P3[:nx, nx].copy()
    Y, y = {}, {}
    for w in range(nseg - 2, -1, -1):
        V = segs[w][0][st[w]]
        Vxx, Vx1, Vxl = V[:nx, :nx], V[:nx, nx], V[:nx, L:]
        Vll, Vl1, Vlx = V[L:, L:], V[L:, nx], V[L:, :nx]
        T = np.eye(nx) - Ph @ Vll
        Y[w] = np.linalg.solve(T, Ph @ Vlx)
        y[w] = np.linalg.solve(T, Ph @ Vl1 + ph)
        Ph, ph = Vxx + Vxl @ Y[w], Vx1 + Vxl @ y[w]
    xh = [np.zeros(nx)]
    lam = []
    for w in range(nseg - 1):
        V = segs[w][0][st[w]]
        Vll, Vl1, Vlx = V[L:, L:], V[L:, nx], V[L:, :nx]
        lam.append(Y[w] @ xh[w] + y[w])
        xh.append(Vlx @ xh[w] + Vl1 + Vll @ lam[w])
    lam.append(np.zeros(nx))
    # forward sweeps per segment
    out = np.zeros((H + 1, nx + nu))
    for w in range(nseg):
        x = xh[w].copy()
        for k in range(st[w], st[w + 1]):
            Kp = segs[w][1][k]
            u = Kp[:, :nx] @ x + Kp[:, nx] + Kp[:, nx + 1:] @ lam[w]
            out[k, :nx], out[k, nx:] = x, u
            x = A[k] @ x + B[k] @ u + c[k]
        if w == nseg - 1:
            out[H, :nx] = x
        else:
            assert np.allclose(x, xh[w + 1], atol=1e-9), (w, x, xh[w + 1])
    return out, segs, st, lam, xh


def corrector_check(A, B, c, h, g, H, nx, nu, segs, st, nseg=4):
    """Factor fixed: the segment's p (lambda-free) and V_l1 from the vector recursions equal the
    CI column of a fresh augmented factorisation with the new gradient g."""
    L = nx + 1
    for w in range(nseg):
        Ps, Ks, Rui = segs[w]
        a0, b0, last = st[w], st[w + 1], w == nseg - 1
        Pf, Kf, _ = seg_factor(A, B, c, h, g, a0, b0, last, nx, nu, H)
        p = g[H][:nx].copy() if last else np.zeros(nx)
        Vl1 = np.zeros(nx)
        for k in range(b0 - 1, a0 - 1, -1):
            Pn = np.zeros((nx, nx)) if (not last and k + 1 == b0) else Ps[k + 1][:nx, :nx]
            t = Pn @ c[k]
            Kx = Ks[k][:, :nx]
            kff = -Rui[k] @ (g[k][nx:] + B[k].T @ (t + p))
            Acl = A[k] + B[k] @ Kx
            p = g[k][:nx] + Kx.T @ g[k][nx:] + Acl.T @ t + Acl.T @ p
            assert np.allclose(kff, Kf[k][:, nx], atol=1e-9)
            assert np.allclose(p, Pf[k][:nx, nx], atol=1e-9), (w, k)
            Plx = np.eye(nx) if (not last and k + 1 == b0) else Ps[k + 1][L:, :nx]
            Vl1 += Plx @ (c[k] + B[k] @ kff)
        if not last:
            assert np.allclose(Vl1, Pf[a0][L:, nx], atol=1e-9), w


def main():
    rng = np.random.default_rng(0)
    for (nx, nu, H) in [(4, 1, 20), (6, 2, 30), (4, 1, 10), (6, 2, 8)]:
        A = [np.eye(nx) + 0.1 * rng.standard_normal((nx, nx)) for _ in range(H)]
        B = [0.3 * rng.standard_normal((nx, nu)) for _ in range(H)]
        c = [0.1 * rng.standard_normal(nx) for _ in range(H)]
        h = [np.exp(rng.standard_normal(nx + nu)) for _ in range(H + 1)]
        g = [rng.standard_normal(nx + nu) for _ in range(H + 1)]
        ref = kkt_solve(A, B, c, h, g, H, nx, nu)
        out, segs, st, lam, xh = seg_solve(A, B, c, h, g, H, nx, nu)
        err = np.abs(out[:, :] - ref[:, :]).max()
        ref[H, nx:] = 0.0
        print(f"nx={nx} nu={nu} H={H}: |w_seg - w_kkt| = {np.abs(out - ref).max():.2e}")
        assert np.abs(out - ref).max() < 1e-9, err
        g2 = [rng.standard_normal(nx + nu) for _ in range(H + 1)]
        corrector_check(A, B, c, h, g2, H, nx, nu, segs, st)
    print("ok")


if __name__ == "__main__":
    main()
