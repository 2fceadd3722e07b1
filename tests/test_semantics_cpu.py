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
