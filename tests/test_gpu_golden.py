"""The HIP path against the reference-generated golden vectors directly (MI355X only).

tests/golden/golden_quad3d.npz holds outputs of the reference's own functions (made by
tests/golden/make_golden.py with casadi/gpytorch/acados stand-ins and the exact GP posterior); the
CPU tests pin the oracle to them (tests/test_oracle_golden.py), the other GPU tests compare the GPU
with the oracle.  These tests skip the oracle: GPU outputs against the fixture itself.

* GP mean at the golden query points (`gpytorch_predict2casadi`, `gpmpc/gp.py:72-85`) through both
  GPU paths: the linearisation's MFMA tile sums (`gpmpc_gp_mean_grad`) and the posterior kernel
  (`GaussianProcess.predict`).
* `propagate_constraint_limits` (`gpmpc/gpmpc.py:425-498`): the per-stage tightening the SQP kernel
  computes from the previous solution set to the fixture's x_prev / u_prev, with the fixture's GPs
  and LQR gain, against the reference's output.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GP_IDX = [[0], [1, 2, 3], [4, 5, 6]]


def _torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _golden_gps(g, torch):
    from gpmpc.gp import GaussianProcess

    gps = []
    for i, idx in enumerate(GP_IDX):
        gp = GaussianProcess(torch.tensor(g["gp_Xtr"][:, idx]), torch.tensor(g["gp_Ytr"][:, i]))
        gp.set_hyperparameters(*g["gp_hyp"][i])
        gps.append(gp)
    return gps


def test_gp_mean_matches_reference_fixture(golden3d):
    torch = _torch()
    from gpmpc.models import quad3d_spec
    from gpmpc.solver import BatchSolver

    g = golden3d
    gps = _golden_gps(g, torch)
    solver = BatchSolver(quad3d_spec(), 10, 1)
    solver.set_gps(gps)
    for i, idx in enumerate(GP_IDX):
        zq = torch.tensor(g["gp_Zq"][:, idx])
        ref = g[f"gp{i}_mean_q"]
        # absolute scale of the mean's terms: sf2 sum |alpha| (K is ill-conditioned, the fixture's
        # K^-1 y and the build's Cholesky solve agree to that scale, as in test_oracle_golden)
        alpha = torch.cholesky_solve(torch.tensor(g["gp_Ytr"][:, i])[:, None],
                                     torch.linalg.cholesky(torch.tensor(g[f"gp{i}_K"])))[:, 0]
        scale = float(g["gp_hyp"][i][1]) * float(alpha.abs().sum())
        mean_lin, _ = solver.gp_mean_grad(i, zq)
        np.testing.assert_allclose(mean_lin.cpu().numpy(), ref, rtol=0, atol=1e-12 * scale)
        mean_post, _ = gps[i].predict(zq.cuda(), return_var=False)
        np.testing.assert_allclose(mean_post.cpu().numpy(), ref, rtol=0, atol=1e-12 * scale)


def test_tightening_matches_reference_fixture(golden3d):
    torch = _torch()
    from gpmpc.models import quad3d_spec
    from gpmpc.solver import BatchSolver

    g = golden3d
    spec = quad3d_spec()   # the reference's variance-input map (variance at z[:, gp_idx])
    H = g["tt_x_prev"].shape[1] - 1
    solver = BatchSolver(spec, H, 1)
    solver.set_gps(_golden_gps(g, torch))
    solver.set_tightening(True, float(g["tt_prob"]), g["lqr_Ad"], g["lqr_Bd"], g["lqr_K"])
    solver.reset(reset_iterate=True)
    # one solve from hover marks a previous solution; the iterate is then replaced by the fixture's
    x0 = torch.zeros(1, spec.nx, dtype=torch.float64, device="cuda")
    x0[0, 4] = 1.0
    ts = torch.zeros(1, dtype=torch.int32, device="cuda")
    solver.solve(x0, ts)
    assert int(solver.status[0]) in (0, 2)
    xp = torch.tensor(g["tt_x_prev"].T[None].copy(), device="cuda")
    up = torch.tensor(g["tt_u_prev"].T[None].copy(), device="cuda")
    solver.set_iterate(xp, up)
    solver.solve(x0, ts)              # variance launch at (x_prev, u_prev), tightening in the SQP kernel
    tight = solver.solution()[2].cpu().numpy()[0]          # (H + 1, nx + nu): icdf sqrt(var) per variable
    sc, ic = g["tt_state"], g["tt_input"]                  # reference: (2 nx, H + 1), (2 nu, H)
    nx, nu = spec.nx, spec.nu
    np.testing.assert_allclose(tight[:, :nx], -sc[:nx].T, rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(tight[:, :nx], -sc[nx:].T, rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(tight[:H, nx:], -ic[:nu].T, rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(tight[:H, nx:], -ic[nu:].T, rtol=1e-9, atol=1e-13)
