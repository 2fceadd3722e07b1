"""The C++ CPU restatement (oracle/cpu_ref.cpp, bench.py's CPU baseline) against the numpy
oracle: closed loop with tightening, both at KKT tolerance 1e-9, trajectories within
1e-7 (1 + |x|).  Same algorithm, different linear algebra (Riccati vs dense KKT)."""

import numpy as np
import pytest

from helpers import O, initial_states, lqr, oracle_gps, oracle_step, problem


def _cpu_ref():
    from oracle import cpu_ref

    if not cpu_ref.LIB_PATH.exists():
        pytest.skip("oracle/lib/libcpuref.so not built (make -C oracle)")
    return cpu_ref


@pytest.mark.parametrize("name,N,H,B,steps,love", [("quad2d", 40, 20, 2, 3, False), ("cartpole", 30, 15, 2, 3, False),
                                                    ("quad3d", 60, 15, 1, 2, False), ("quad2d", 60, 20, 2, 3, True)])
def test_cpu_ref_matches_numpy_oracle(name, N, H, B, steps, love):
    """love: both sides take the tightening variance from the same rank-20 LOVE root
    (cpuref_set_gp_var_root vs oracle.love_var), the bench's CPU baseline for configs 4/5."""
    cpu_ref = _cpu_ref()
    spec, data, hyp = problem(name, N)
    gpo = oracle_gps(data, hyp)
    mats = lqr(spec)
    tol = 1e-9
    roots = None
    if love:
        rng = np.random.default_rng(5)
        roots = [O.lanczos_love_root(og.K, 20, rng.standard_normal(N)) for og in gpo]
        for og, R in zip(gpo, roots):
            og.var = (lambda Z, with_noise=True, og=og, R=R: O.love_var(og, R, Z, with_noise))
    ref = cpu_ref.CpuRef(spec, H, B, gps=gpo, lqr_mats=mats, tol=tol, qp_tol=1e-11, qp_max_iter=100,
                         love_roots=roots)
    zr = np.random.default_rng(9)
    for g, og in enumerate(gpo):   # the variance itself (the closed loop barely feels the tightening)
        Z = og.X[zr.integers(0, N, 40)] + 0.3 * zr.standard_normal((40, og.X.shape[1]))
        np.testing.assert_allclose(ref.gp_var(g, Z), og.var(Z, with_noise=True), rtol=0, atol=1e-12 * og.sf2)
    sd = spec.to_dict()
    opts = O.SQPOptions(tol_stat=tol, tol_eq=tol, tol_ineq=tol, tol_comp=tol, qp_tol=1e-11, qp_max_iter=100)
    orc = [O.SQPSolver(sd, O.Dynamics(sd, gpo), H, opts) for _ in range(B)]
    plant = O.Dynamics(sd, None, params=spec.true_params)
    traj = spec.reference_trajectory()
    x0, phase = initial_states(spec, traj, B)
    prev = [None] * B
    for step in range(steps):
        u0 = ref.step(x0, phase + step, threads=2).copy()
        for b in range(B):
            so, _, _ = oracle_step(spec, orc[b], gpo, x0[b], int(phase[b]) + step, H, traj, prev[b], lqr_mats=mats)
            assert ref.status[b] == so == 0, (step, b, ref.status[b], so)
            ex = np.abs(ref.x[b] - orc[b].x).max() / (1 + np.abs(orc[b].x).max())
            eu = np.abs(ref.u[b] - orc[b].u).max() / (1 + np.abs(orc[b].u).max())
            assert max(ex, eu) <= 1e-7, (step, b, ex, eu)
            prev[b] = (orc[b].x.T.copy(), orc[b].u.T.copy())
            x0[b] = plant.rk4(x0[b], u0[b])[0]
