#!/usr/bin/env python3
"""Numpy model of the two-segment Newton solve of sqp_kernel.hip (SqpKernel::kSeg), in the kernel's
16-slot tile layout, against the dense KKT solve.

The IPM's Newton system is the LQ problem over stages 0..H with dx_0 = 0:
    min sum_k 1/2 w_k' diag(h_k) w_k + g_k' w_k,   dx_{k+1} = A_k dx_k + B_k du_k + c_k.
Segment A = stages 0..m-1 runs the Riccati recursion over z = [x; 1; lambda] from the terminal
cost lambda' x_m (lambda: the unknown costate of x_m), segment B = stages m..H-1 the ordinary one
from the true P_H; both are the kernel's 5-MFMA stage (tile slots x 0..NX-1, CI = NX, u 8..,
lambda 8+NU..): W' = P'[:, 0:8] G''[0:8, :] + (lambda columns of P'), M' = G''[0:8, :]' W'[0:8, :]
+ C with C = D outside the lambda rows and the lambda rows of W' inside, P' <- M' + M'_{.u} K'.
Then the boundary: T = I - Ph V_ll (Ph, ph: segment B's cost-to-go at m), lambda = T^-1 (Ph V_l1
+ ph) (Gauss-Jordan with partial pivoting), x_m = V_l1 + V_ll lambda; forward sweeps of both
segments (segment A with kff + K_lambda lambda).  Also the corrector (factorisation fixed, new
gradient): zero-terminal p recursion on A, V_l1 = sum P_lx,k+1 (c_k + B_k kff_k).

    python tools/seg2_proto.py
"""

import numpy as np


def kkt_solve(A, B, c, h, g, H, nx, nu):
    nb = nx + nu
    nv = (H + 1) * nb
    ne = (H + 1) * nx
    K = np.zeros((nv + ne, nv + ne))
    rhs = np.zeros(nv + ne)
    for k in range(H + 1):
        K[k * nb:(k + 1) * nb, k * nb:(k + 1) * nb] = np.diag(h[k])
        rhs[k * nb:(k + 1) * nb] = -g[k]
    for i in range(nx):
        K[nv + i, i] = K[i, nv + i] = 1.0
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
    w = sol[:nv].reshape(H + 1, nb)
    pi = sol[nv + nx:].reshape(H, nx)     # multipliers of the dynamics rows
    return w, pi


def slots(nx, nu):
    CI, UI = nx, 8
    LI = UI + nu
    assert LI + nx <= 16
    return CI, UI, LI


def stage_tile(P, A, B, c, h, g, nx, nu, aug):
    """One factorisation stage in the tile algebra; returns P'_k (16x16), K' row block (nu x 16), Ru^-1."""
    CI, UI, LI = slots(nx, nu)
    G = np.zeros((16, 16))            # G''[k][n]: rows x_next / CI / lambda, columns x / CI / u / lambda
    G[:nx, :nx] = A
    G[:nx, CI] = c
    G[:nx, UI:UI + nu] = B
    G[CI, CI] = 1.0
    lam = np.zeros(16, bool)
    lam[LI:LI + nx] = aug
    D = np.zeros((16, 16))
    for i in range(nx):
        D[i, i] = h[i]
        D[i, CI] = D[CI, i] = g[i]
    for a in range(nu):
        D[UI + a, UI + a] = h[nx + a]
        D[UI + a, CI] = D[CI, UI + a] = g[nx + a]
    Cw = np.where(lam[None, :], P, 0.0)                 # W' C-init: P's lambda columns
    W = P[:, 0:8] @ G[0:8, :] + Cw                      # 2 MFMAs (K = 0..7)
    Cm = np.where(lam[:, None], W, D)                   # M' C-init: lambda rows of W', else D
    M = G[0:8, :].T @ W[0:8, :] + Cm                    # 2 MFMAs
    Ru = M[UI:UI + nu, UI:UI + nu]
    Ri = np.linalg.inv(Ru)
    Kp = -Ri @ M[UI:UI + nu, :]                         # all 16 columns (K, kff, K_lambda)
    Pn = M + M[:, UI:UI + nu] @ Kp                      # 1 MFMA
    return Pn, Kp, Ri


def factor(A, B, c, h, g, k0, k1, aug, nx, nu, H):
    CI, UI, LI = slots(nx, nu)
    P = np.zeros((16, 16))
    if not aug:   # true terminal cost of stage H
        P[:nx, :nx] = np.diag(h[H][:nx])
        P[:nx, CI] = P[CI, :nx] = g[H][:nx]
    else:         # lambda' x_m
        for i in range(nx):
            P[i, LI + i] = P[LI + i, i] = 1.0
    Ps, Ks, Rs = {k1: P.copy()}, {}, {}
    for k in range(k1 - 1, k0 - 1, -1):
        P, Kp, Ri = stage_tile(P, A[k], B[k], c[k], h[k], g[k], nx, nu, aug)
        Ps[k], Ks[k], Rs[k] = P.copy(), Kp, Ri
    return Ps, Ks, Rs


def gauss_jordan(M, nrows):
    """[T | rhs...] -> [I | T^-1 rhs...] with partial pivoting, column per 'lane'."""
    M = M.copy()
    for p in range(nrows):
        piv = p + int(np.argmax(np.abs(M[p:, p])))
        M[[p, piv]] = M[[piv, p]]
        M[p] /= M[p, p]
        for i in range(nrows):
            if i != p:
                M[i] -= M[i, p] * M[p]
    return M


def seg2_solve(A, B, c, h, g, H, nx, nu, m):
    CI, UI, LI = slots(nx, nu)
    PA, KA, RA = factor(A, B, c, h, g, 0, m, True, nx, nu, H)
    PB, KB, RB = factor(A, B, c, h, g, m, H, False, nx, nu, H)
    V = PA[0]
    Vll, Vl1 = V[LI:LI + nx, LI:LI + nx], V[LI:LI + nx, CI]
    Ph, ph = PB[m][:nx, :nx], PB[m][:nx, CI]
    T = np.eye(nx) - Ph @ Vll
    Mg = np.hstack([T, (Ph @ Vl1 + ph)[:, None], np.eye(nx)])
    R = gauss_jordan(Mg, nx)
    lam, Tinv = R[:, nx], R[:, nx + 1:]
    xm = Vl1 + Vll @ lam
    out = np.zeros((H + 1, nx + nu))
    pi = np.zeros((H, nx))
    x = np.zeros(nx)
    K, P = {**KA, **KB}, {**PA, **PB}
    P[m] = PB[m]                      # the true cost-to-go at m (segment B's start)
    for k in range(H):
        if k == m:
            assert np.allclose(x, xm, atol=1e-9), (x, xm)
            x = xm
        Kp = K[k]
        u = Kp[:, :nx] @ x + Kp[:, CI]
        if k < m:
            u = u + Kp[:, LI:LI + nx] @ lam
        out[k, :nx], out[k, nx:] = x, u
        x = A[k] @ x + B[k] @ u + c[k]
    out[H, :nx] = x
    for k in range(H):   # dpi_k = -(P_{k+1} dx_{k+1} + p_{k+1} (+ P_x,lambda lambda inside segment A: the
                         # kernel folds it into p_{k+1}, seg_fold)
        Pn = P[k + 1]
        v = Pn[:nx, :nx] @ out[k + 1, :nx] + Pn[:nx, CI]
        if k + 1 < m:
            v = v + Pn[:nx, LI:LI + nx] @ lam
        pi[k] = -v
    return out, pi, (PA, KA, RA, PB, KB, RB, Ph, Tinv)


def corrector_check(A, B, c, h, g2, H, nx, nu, m, fac):
    """Factorisation fixed, new gradient g2: zero-terminal p recursion on A, V_l1 = sum_k P_lx,k+1 (c_k
    + B_k kff_k), the boundary with the stored T^-1 / Ph, then the same forward / recovery."""
    CI, UI, LI = slots(nx, nu)
    PA, KA, RA, PB, KB, RB, Ph, Tinv = fac
    ref, rpi = kkt_solve(A, B, c, h, g2, H, nx, nu)

    def vec_backward(k0, k1, P, K, R, last):
        p = g2[H][:nx].copy() if last else np.zeros(nx)
        pk, kff = {k1: p.copy()}, {}
        for k in range(k1 - 1, k0 - 1, -1):
            Pn = np.zeros((nx, nx)) if (not last and k + 1 == k1) else P[k + 1][:nx, :nx]
            t = Pn @ c[k]
            Kx = K[k][:, :nx]
            kf = -R[k] @ (g2[k][nx:] + B[k].T @ (t + p))
            Acl = A[k] + B[k] @ Kx
            p = g2[k][:nx] + Kx.T @ g2[k][nx:] + Acl.T @ t + Acl.T @ p
            pk[k], kff[k] = p.copy(), kf
        return pk, kff

    pA, kA = vec_backward(0, m, PA, KA, RA, False)
    pB, kB = vec_backward(m, H, PB, KB, RB, True)
    Vl1 = np.zeros(nx)
    for k in range(m):
        Plx = np.eye(nx) if k + 1 == m else PA[k + 1][LI:LI + nx, :nx]
        Vl1 += Plx @ (c[k] + B[k] @ kA[k])
    lam = Tinv @ (Ph @ Vl1 + pB[m])
    Vll = PA[0][LI:LI + nx, LI:LI + nx]
    xm = Vl1 + Vll @ lam
    x = np.zeros(nx)
    out = np.zeros((H + 1, nx + nu))
    for k in range(H):
        if k == m:
            assert np.allclose(x, xm, atol=1e-9)
        if k < m:
            Kp = KA[k]
            u = Kp[:, :nx] @ x + kA[k] + Kp[:, LI:LI + nx] @ lam
        else:
            u = KB[k][:, :nx] @ x + kB[k]
        out[k, :nx], out[k, nx:] = x, u
        x = A[k] @ x + B[k] @ u + c[k]
    out[H, :nx] = x
    r = ref.copy()
    r[H, nx:] = 0.0
    err = np.abs(out - r).max()
    pi = np.zeros((H, nx))
    for k in range(H):
        if k + 1 < m:
            v = PA[k + 1][:nx, :nx] @ out[k + 1, :nx] + pA[k + 1] + PA[k + 1][:nx, LI:LI + nx] @ lam
        else:
            v = PB[k + 1][:nx, :nx] @ out[k + 1, :nx] + pB[k + 1]
        pi[k] = -v
    return err, np.abs(pi - rpi).max()


def main():
    rng = np.random.default_rng(0)
    for (nx, nu, H) in [(6, 2, 30), (4, 1, 20), (6, 2, 12), (4, 1, 10), (6, 2, 31)]:
        A = [np.eye(nx) + 0.1 * rng.standard_normal((nx, nx)) for _ in range(H)]
        B = [0.3 * rng.standard_normal((nx, nu)) for _ in range(H)]
        c = [0.1 * rng.standard_normal(nx) for _ in range(H)]
        h = [np.exp(rng.standard_normal(nx + nu)) for _ in range(H + 1)]
        g = [rng.standard_normal(nx + nu) for _ in range(H + 1)]
        ref, rpi = kkt_solve(A, B, c, h, g, H, nx, nu)
        ref[H, nx:] = 0.0
        for m in (H // 2, 1, H - 1):
            out, pi, fac = seg2_solve(A, B, c, h, g, H, nx, nu, m)
            e, ep = np.abs(out - ref).max(), np.abs(pi - rpi).max()
            g2 = [rng.standard_normal(nx + nu) for _ in range(H + 1)]
            ec, epc = corrector_check(A, B, c, h, g2, H, nx, nu, m, fac)
            print(f"nx={nx} nu={nu} H={H} m={m}: predictor |w - w_kkt| {e:.1e} |pi - pi_kkt| {ep:.1e}; "
                  f"corrector {ec:.1e} / {epc:.1e}")
            assert max(e, ep, ec, epc) < 1e-9
    print("ok")


if __name__ == "__main__":
    main()
