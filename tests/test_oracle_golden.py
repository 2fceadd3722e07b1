"""The CPU oracle against golden vectors produced by the reference's own functions.

Fixtures: tests/golden/golden_quad3d.npz, made by tests/golden/make_golden.py from
/root/reference (casadi/gpytorch/acados replaced by stand-ins; exact GP posterior).
"""

import numpy as np

from oracle import gpmpc_oracle as O


def test_se_kernel_matches_covSE(golden3d):
    g = golden3d
    k = O.se_kernel(g["k_z"][None], g["k_X"], float(g["k_ell"]), float(g["k_sf2"]))[0]
    np.testing.assert_allclose(k, g["k_single"], rtol=1e-14, atol=0)
    np.testing.assert_allclose(k, g["k_vec"], rtol=1e-14, atol=0)


def test_exact_gp_covariances_and_mean(golden3d):
    g = golden3d
    gp_idx = [[0], [1, 2, 3], [4, 5, 6]]
    for i, idx in enumerate(gp_idx):
        ell, sf2, sn2 = g["gp_hyp"][i]
        gp = O.ExactGP(g["gp_Xtr"][:, idx], g["gp_Ytr"][:, i], ell, sf2, sn2)
        np.testing.assert_allclose(gp.K, g[f"gp{i}_K"], rtol=1e-13, atol=1e-13)
        # K_inv of an ill-conditioned K: compare through K K_inv = I
        np.testing.assert_allclose(gp.K @ g[f"gp{i}_Kinv"], np.eye(len(gp.y)), atol=1e-6)
        m = gp.mean(g["gp_Zq"][:, idx])
        scale = np.abs(gp.alpha).sum() * sf2
        np.testing.assert_allclose(m, g[f"gp{i}_mean_q"], rtol=0, atol=1e-12 * scale)


def test_prior_lqr(golden3d):
    g = golden3d
    Q = np.diag(np.array([8, 0.1, 8, 0.1, 8, 0.1, 0.5, 0.5, 0.5, 0.001, 0.001, 0.001]))
    R = np.diag(np.array([3, 3, 3, 0.1]))
    Ad, Bd, K = O.setup_prior_dynamics(g["lqr_dfdx"], g["lqr_dfdu"], Q, R, 0.02)
    np.testing.assert_allclose(Ad, g["lqr_Ad"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(Bd, g["lqr_Bd"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(K, g["lqr_K"], rtol=1e-8, atol=1e-10)


def test_tightening_matches_reference(golden3d):
    g = golden3d
    from gpmpc.models import quad3d_spec

    spec = quad3d_spec().to_dict()
    gp_idx = [[0], [1, 2, 3], [4, 5, 6]]
    gps = [O.ExactGP(g["gp_Xtr"][:, idx], g["gp_Ytr"][:, i], *g["gp_hyp"][i]) for i, idx in enumerate(gp_idx)]
    assert abs(O.inverse_cdf(float(g["tt_prob"]), 12) - float(g["tt_icdf"])) < 1e-14
    sc, ic = O.propagate_constraint_limits(spec, gps, g["tt_x_prev"], g["tt_u_prev"], g["lqr_Ad"], g["lqr_Bd"],
                                           g["lqr_K"], float(g["tt_prob"]))
    np.testing.assert_allclose(sc, g["tt_state"], rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(ic, g["tt_input"], rtol=1e-9, atol=1e-13)


def test_reference_window_and_constraint_rows(golden3d):
    g = golden3d
    w = O.reference_window(g["ref_traj"], int(g["ref_step"]), 10)
    np.testing.assert_array_equal(w, g["ref_window"])
    from gpmpc.models import quad3d_spec

    s = quad3d_spec()
    sym = g["cstr_sym"]
    rows = np.concatenate([-sym + s.x_lo, sym - s.x_hi])
    np.testing.assert_allclose(rows, g["cstr_rows"], rtol=0, atol=1e-15)
