"""Full-size checks at the BASELINE.json configurations that the other parity tests run small.

* config 3 (north star: quad2d, N=200, H=30, B=1024), the bench's own closed loop at the
  default tolerances: every instance-step converges (status 0) with all four NLP residuals
  below 1e-6, for 12 steps from a cold start;
* the same batch at KKT tolerance 1e-9: 32 sampled instances follow the C++ restatement
  (oracle/cpu_ref.cpp) on the same observations -- same status, |x_gpu - x_cpu| <= 1e-6 (1+|x|);
* the same batch at the shipped options (NLP tolerance 1e-6, QP tolerance = NLP tolerance, mu0 = 1,
  <= 25 SQP iterations) on both sides: 32 sampled instances, same status, trajectories and stage
  costs within the north-star 1e-4 relative;
* config 5 at full size (quad3d, FITC mean on M=2000 inducing rows, exact variance over N=4000,
  H=40): 4 instances x 2 closed-loop steps against the C++ restatement at KKT tolerance 1e-9.
  Reference: `gpmpc/gpmpc.py:377-400` (FITC), `:425-498` (tightening), `:334-368` (select_action).
"""

import numpy as np
import pytest

from helpers import O, fitc_weights, initial_states, lqr, oracle_gps, problem, product_gps

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _cpu_ref():
    from oracle import cpu_ref

    if not cpu_ref.LIB_PATH.exists():
        pytest.skip("oracle/lib/libcpuref.so not built")
    return cpu_ref


def test_config3_full_batch_converges_at_default_tolerances():
    torch = _torch()
    from gpmpc.solver import BatchSolver

    spec, data, hyp = problem("quad2d", 200)
    H, B, steps = 30, 1024, 12
    gs = BatchSolver(spec, H, B)
    gs.set_gps(product_gps(data, hyp))
    gs.set_tightening(True, 0.95, *lqr(spec))
    gs.reset(reset_iterate=True)
    x0, ph = initial_states(spec, spec.reference_trajectory(), B, seed=1)
    obs = torch.tensor(x0, device="cuda")
    ts = torch.tensor(ph, dtype=torch.int32, device="cuda")
    for k in range(steps):
        u = gs.solve(obs, ts)
        st = gs.status.cpu().numpy()
        res = gs.res.cpu().numpy()
        assert (st == 0).all(), (k, np.bincount(st, minlength=5))
        assert res.max() <= 1e-6, (k, res.max(axis=0))
        assert torch.isfinite(u).all()
        gs.plant_step(obs, u, ts, out=obs)


def test_config2_full_batch_converges_at_default_tolerances():
    """Config 2 (cartpole, N=50, H=20, B=256) at the bench defaults and the automatic launch shape
    (four waves per instance: B <= CUs): every instance-step converges with all four NLP residuals
    below 1e-6 over 12 closed-loop steps from a cold start."""
    torch = _torch()
    from gpmpc.solver import BatchSolver

    spec, data, hyp = problem("cartpole", 50)
    H, B, steps = 20, 256, 12
    gs = BatchSolver(spec, H, B)
    gs.set_gps(product_gps(data, hyp))
    gs.set_tightening(True, 0.95, *lqr(spec))
    gs.reset(reset_iterate=True)
    x0, ph = initial_states(spec, spec.reference_trajectory(), B, seed=1)
    obs = torch.tensor(x0, device="cuda")
    ts = torch.tensor(ph, dtype=torch.int32, device="cuda")
    for k in range(steps):
        u = gs.solve(obs, ts)
        st = gs.status.cpu().numpy()
        res = gs.res.cpu().numpy()
        assert (st == 0).all(), (k, np.bincount(st, minlength=5))
        assert res.max() <= 1e-6, (k, res.max(axis=0))
        assert torch.isfinite(u).all()
        gs.plant_step(obs, u, ts, out=obs)


def test_config4_full_batch_converges_with_love_variance():
    """Config 4 per GPU (quad2d, N=1000, H=30, B=1024) at the bench defaults: the tightening
    variance from the LOVE roots (gpytorch fast_pred_var above 800 rows, `gpmpc/gpmpc.py:441-445`);
    every instance-step converges with all NLP residuals <= 1e-6 over 6 closed-loop steps."""
    torch = _torch()
    from gpmpc.solver import BatchSolver

    spec, data, hyp = problem("quad2d", 1000)
    H, B, steps = 30, 1024, 6
    gs = BatchSolver(spec, H, B)
    gs.set_gps(product_gps(data, hyp), variance="love")
    assert all(r is not None for r in gs.love_ranks), gs.love_ranks
    gs.set_tightening(True, 0.95, *lqr(spec))
    gs.reset(reset_iterate=True)
    x0, ph = initial_states(spec, spec.reference_trajectory(), B, seed=1)
    obs = torch.tensor(x0, device="cuda")
    ts = torch.tensor(ph, dtype=torch.int32, device="cuda")
    for k in range(steps):
        u = gs.solve(obs, ts)
        st = gs.status.cpu().numpy()
        res = gs.res.cpu().numpy()
        assert (st == 0).all(), (k, np.bincount(st, minlength=5))
        assert res.max() <= 1e-6, (k, res.max(axis=0))
        assert torch.isfinite(u).all()
        if k >= 1:
            assert gs.solution()[2].cpu().numpy()[:, 1:, :].max() > 0.0   # tightening active
        gs.plant_step(obs, u, ts, out=obs)


def test_config3_full_batch_sampled_instances_match_cpp_restatement():
    torch = _torch()
    cpu_ref = _cpu_ref()
    from gpmpc.solver import BatchSolver

    spec, data, hyp = problem("quad2d", 200)
    H, B, steps, tol = 30, 1024, 10, 1e-9
    mats = lqr(spec)
    gs = BatchSolver(spec, H, B, tol=tol, qp_tol=1e-11, qp_max_iter=100)
    gs.set_gps(product_gps(data, hyp))
    gs.set_tightening(True, 0.95, *mats)
    gs.reset(reset_iterate=True)
    sample = np.random.default_rng(3).choice(B, 32, replace=False)
    ref = cpu_ref.CpuRef(spec, H, len(sample), gps=oracle_gps(data, hyp), lqr_mats=mats, tol=tol, qp_tol=1e-11,
                         qp_max_iter=100)
    x0, ph = initial_states(spec, spec.reference_trajectory(), B, seed=1)
    obs = torch.tensor(x0, device="cuda")
    ts = torch.tensor(ph, dtype=torch.int32, device="cuda")
    for k in range(steps):
        xo = obs.cpu().numpy()
        u = gs.solve(obs, ts)
        st = gs.status.cpu().numpy()
        assert (st == 0).mean() >= 0.95, (k, np.bincount(st, minlength=5))
        ref.step(xo[sample].copy(), ph[sample] + k, threads=8)
        np.testing.assert_array_equal(st[sample], ref.status)
        xg = gs.solution()[0].cpu().numpy()[sample]
        ok = ref.status == 0
        err = np.abs(xg - ref.x).max(axis=(1, 2)) / (1 + np.abs(ref.x).max(axis=(1, 2)))
        assert err[ok].max() <= 1e-6, (k, err[ok].max())
        gs.plant_step(obs, u, ts, out=obs)


def test_config3_shipped_defaults_match_cpp_restatement_with_stage_costs():
    """Config 3 (quad2d, N=200, H=30, B=1024) with both sides at the shipped options -- NLP
    tolerance 1e-6 (acados default), QP tolerance = NLP tolerance (acados passes its NLP tolerances
    to the QP solver when the OCP sets none, `gpmpc/gpmpc.py:257-263`), mu0 = 1, <= 25 SQP iterations:
    32 sampled instances over 10 closed-loop steps on the GPU's observations, identical status,
    x, u within 1e-4 (1 + |.|) (the north-star tolerance) and the per-stage LINEAR_LS costs
    (`gpmpc/gpmpc.py:231-239`, gpmpc_set_cost_buffer) within 1e-4 of the total cost."""
    torch = _torch()
    cpu_ref = _cpu_ref()
    from gpmpc.solver import BatchSolver

    spec, data, hyp = problem("quad2d", 200)
    H, B, steps = 30, 1024, 10
    mats = lqr(spec)
    gs = BatchSolver(spec, H, B)                                  # shipped defaults
    gs.set_gps(product_gps(data, hyp))
    gs.set_tightening(True, 0.95, *mats)
    gs.reset(reset_iterate=True)
    gs.set_cost_output(True)
    sample = np.random.default_rng(3).choice(B, 32, replace=False)
    ref = cpu_ref.CpuRef(spec, H, len(sample), gps=oracle_gps(data, hyp), lqr_mats=mats)   # same defaults
    traj, sd = spec.reference_trajectory(), spec.to_dict()
    x0, ph = initial_states(spec, traj, B, seed=1)
    obs = torch.tensor(x0, device="cuda")
    ts = torch.tensor(ph, dtype=torch.int32, device="cuda")
    worst = 0.0
    for k in range(steps):
        xo = obs.cpu().numpy()
        u = gs.solve(obs, ts)
        st = gs.status.cpu().numpy()
        ref.step(xo[sample].copy(), ph[sample] + k, threads=8)
        np.testing.assert_array_equal(st[sample], ref.status)
        assert (ref.status == 0).all(), (k, ref.status)
        xg, ug, _ = (t.cpu().numpy()[sample] for t in gs.solution())
        ex = np.abs(xg - ref.x).max(axis=(1, 2)) / (1 + np.abs(ref.x).max(axis=(1, 2)))
        eu = np.abs(ug - ref.u).max(axis=(1, 2)) / (1 + np.abs(ref.u).max(axis=(1, 2)))
        assert max(ex.max(), eu.max()) <= 1e-4, (k, ex.max(), eu.max())
        cost = gs.stage_cost.cpu().numpy()[sample]
        for i, b in enumerate(sample):
            co = O.stage_costs(sd, ref.x[i], ref.u[i], traj, ph[b] + k)
            cg = O.stage_costs(sd, xg[i], ug[i], traj, ph[b] + k)
            np.testing.assert_allclose(cost[i], cg, rtol=1e-12, atol=1e-15)     # the kernel's costs
            np.testing.assert_allclose(cost[i], co, rtol=0, atol=1e-4 * co.sum())
            worst = max(worst, np.abs(cost[i] - co).max() / co.sum())
        gs.plant_step(obs, u, ts, out=obs)
    print(f"shipped defaults: worst stage-cost difference {worst:.2e} of the total cost")


def test_config5_full_size_matches_cpp_restatement():
    torch = _torch()
    cpu_ref = _cpu_ref()
    from gpmpc.solver import BatchSolver

    spec, data, hyp = problem("quad3d", 4000)
    spec.var_inputs = spec.gp_inputs                     # bench config 5: variance at each GP's inputs
    H, B, M, tol = 40, 4, 2000, 1e-9
    gpp = product_gps(data, hyp)
    fitc = fitc_weights(gpp, M)
    mats = lqr(spec)
    gs = BatchSolver(spec, H, B, tol=tol, qp_tol=1e-11, qp_max_iter=100)
    gs.set_var_inputs(spec.var_inputs)
    gs.set_gps(gpp, fitc=fitc)
    gs.set_tightening(True, 0.95, *mats)
    gs.reset(reset_iterate=True)
    ref = cpu_ref.CpuRef(spec, H, B, gps=oracle_gps(data, hyp), lqr_mats=mats, tol=tol, qp_tol=1e-11,
                         qp_max_iter=100, fitc=fitc)
    traj = spec.reference_trajectory()
    x0, ph = initial_states(spec, traj, B)
    plant = O.Dynamics(spec.to_dict(), None, params=spec.true_params)
    for k in range(2):
        gs.solve(torch.tensor(x0, device="cuda"), torch.tensor(ph + k, dtype=torch.int32, device="cuda"))
        u0 = ref.step(x0, ph + k, threads=4).copy()
        st = gs.status.cpu().numpy()
        np.testing.assert_array_equal(st, ref.status)
        assert (st == 0).all(), st
        xg, ug, tg = (t.cpu().numpy() for t in gs.solution())
        err = np.abs(xg - ref.x).max() / (1 + np.abs(ref.x).max())
        assert err <= 1e-6, (k, err)
        if k == 1:
            assert tg[:, 1:, :].max() > 0.0               # the tightening from the N=4000 variance is active
        for b in range(B):
            x0[b] = plant.rk4(x0[b], u0[b])[0]
