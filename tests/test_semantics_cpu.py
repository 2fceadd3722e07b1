"""Host-side semantics of the drop-in classes and the CPU restatements (no GPU):

* ``MPC(q_mpc, r_mpc)`` applies the weights (`gpmpc/mpc.py:42-45`), exposes ``U_EQ``
  (`gpmpc/mpc.py:15`, `gpmpc/gpmpc.py:18`) and never mutates the caller's spec;
* an obs outside the stage-0 state box is an infeasible QP, status 4
  (`gpmpc/gpmpc.py:288,296,309-310`), in both CPU restatements, and a failed solve keeps the
  previous iterate (no poisoning of later steps).
"""

import numpy as np
import pytest

from helpers import O, initial_states, lqr, oracle_gps, oracle_step, problem


def test_mpc_applies_q_r_and_exposes_u_eq():
    from gpmpc.gpmpc import GPMPC
    from gpmpc.models import get_spec
    from gpmpc.mpc import MPC

    spec = get_spec("quad3d")
    q0 = spec.q_diag.copy()
    q = np.arange(1, 13, dtype=float)
    r = np.array([1.0, 2.0, 3.0, 4.0])
    ctrl = MPC(spec, q_mpc=list(q), r_mpc=list(r), horizon=7)     # the GPU handle is built lazily
    np.testing.assert_array_equal(ctrl.model.q_diag, q)
    np.testing.assert_array_equal(ctrl.model.r_diag, r)
    np.testing.assert_array_equal(ctrl.Q, np.diag(q))
    np.testing.assert_array_equal(spec.q_diag, q0)                 # caller's spec untouched
    np.testing.assert_array_equal(MPC.U_EQ, [0.3234, 0, 0, 0])     # gpmpc/mpc.py:15
    np.testing.assert_array_equal(GPMPC.U_EQ, [0.3234, 0, 0, 0])   # gpmpc/gpmpc.py:18
    np.testing.assert_array_equal(ctrl.U_EQ, spec.u_eq)
    np.testing.assert_array_equal(ctrl.u_ref, np.repeat(spec.u_eq[:, None], 7, axis=1))
    q2 = MPC("quad2d", horizon=5)
    np.testing.assert_array_equal(q2.U_EQ, [0.3234, 0.0])
    with pytest.raises(AssertionError):
        MPC("quad2d", q_mpc=[1.0] * 5)


@pytest.mark.parametrize("offset,expect_fail", [(0.0, False), (5e-7, False), (1e-3, True), (np.nan, True)])
def test_oracle_stage0_rows_decide_feasibility(offset, expect_fail):
    spec, data, hyp = problem("quad2d", 40)
    H = 8
    gpo = oracle_gps(data, hyp)
    sd = spec.to_dict()
    sol = O.SQPSolver(sd, O.Dynamics(sd, gpo), H)
    traj = spec.reference_trajectory()
    x0 = initial_states(spec, traj, 1)[0][0]
    st, _, _ = oracle_step(spec, sol, gpo, x0, 0, H, traj, None)
    assert st == 0
    x_prev = sol.x.copy()
    xb = x0.copy()
    # theta (index 4) at its upper bound (GPMPC: hi - 1e-8, uh = -1e-8) plus the offset
    xb[4] = spec.x_hi[4] - 1e-8 + offset
    st, _, _ = oracle_step(spec, sol, gpo, xb, 1, H, traj, None)
    if expect_fail:
        assert st == O.ACADOS_QP_FAILURE
        np.testing.assert_array_equal(sol.x, x_prev)      # previous iterate kept
        assert not sol.pi.any() and not sol.ll.any()
    else:
        assert st in (0, 2)


def test_cpp_restatement_infeasible_obs_is_status_4_and_recovers():
    from oracle import cpu_ref

    if not cpu_ref.LIB_PATH.exists():
        pytest.skip("oracle/lib/libcpuref.so not built")
    spec, data, hyp = problem("quad2d", 40)
    H, B = 8, 3
    ref = cpu_ref.CpuRef(spec, H, B, gps=oracle_gps(data, hyp), lqr_mats=lqr(spec))
    traj = spec.reference_trajectory()
    x0, ph = initial_states(spec, traj, B)
    ref.step(x0, ph)
    assert (ref.status == 0).all()
    x_prev, u_prev = ref.x.copy(), ref.u.copy()
    bad = x0.copy()
    bad[1, 2] = spec.x_hi[2] + 0.1                    # instance 1: z above its box
    bad[2, 0] = np.nan                                # instance 2: NaN observation
    u0 = ref.step(bad, ph + 1).copy()
    assert ref.status[0] == 0 and ref.status[1] == 4 and ref.status[2] == 4
    np.testing.assert_array_equal(ref.x[1:], x_prev[1:])   # failed instances keep their iterate
    np.testing.assert_array_equal(u0[1:], u_prev[1:, 0])   # and return its first input
    assert (ref.has_prev == [1, 0, 0]).all()               # next step untightened, as after a reset
    ref.step(x0, ph + 2)
    assert (ref.status == 0).all() and np.isfinite(ref.x).all()


def test_stage_costs_are_the_linear_ls_objective_of_the_oracle():
    """oracle.stage_costs (acados LINEAR_LS, `gpmpc/gpmpc.py:231-239`: W = blkdiag(Q, R), W_e = Q,
    dt cost scaling on stages 0..T-1) is the objective whose gradient and Gauss-Newton Hessian the
    oracle's SQP uses: d/dw sum_k cost_k = hdiag (w - y_ref), checked by central differences on every
    decision variable of a random trajectory (stage-0 state included: a constant of the QP)."""
    spec, _, _ = problem("quad2d", 10)
    sd = spec.to_dict()
    T, nx, nu = 6, spec.nx, spec.nu
    rng = np.random.default_rng(4)
    traj = spec.reference_trajectory()
    x = traj[:, 3:3 + T + 1].T + 0.1 * rng.standard_normal((T + 1, nx))
    u = spec.u_eq + 0.05 * rng.standard_normal((T, nu))
    sol = O.SQPSolver(sd, O.Dynamics(sd, None), T, O.SQPOptions())
    c = O.stage_costs(sd, x, u, traj, 3)
    assert c.shape == (T + 1,) and (c > 0).all()
    xr = O.reference_window(traj, 3, T).T
    yref = sol._pack(xr, np.repeat(spec.u_eq[None, :], T, axis=0))
    grad = sol.hdiag * (sol._pack(x, u) - yref)          # the oracle's cost gradient over [u_k; x_k+1]
    h = 1e-6
    for j in range(grad.size):
        k, v = divmod(j, nx + nu)
        xp, up, xm, um = x.copy(), u.copy(), x.copy(), u.copy()
        if v < nu:
            up[k, v] += h
            um[k, v] -= h
        else:
            xp[k + 1, v - nu] += h
            xm[k + 1, v - nu] -= h
        fd = (O.stage_costs(sd, xp, up, traj, 3).sum() - O.stage_costs(sd, xm, um, traj, 3).sum()) / (2 * h)
        assert abs(fd - grad[j]) <= 1e-7 * (1 + abs(grad[j])), (j, fd, grad[j])
    # stage 0's state term: dt-scaled Q, like every non-terminal stage
    x2 = x.copy()
    x2[0] += 0.01
    d0 = O.stage_costs(sd, x2, u, traj, 3)[0] - c[0]
    e0 = x[0] - xr[0]
    assert abs(d0 - 0.5 * spec.dt * (((e0 + 0.01) ** 2 - e0 ** 2) @ spec.q_diag)) <= 1e-14
