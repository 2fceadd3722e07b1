"""The default tightening variance of configs 4 and 5 -- the reference's gpytorch
``fast_pred_var`` (LOVE, `gpmpc/gpmpc.py:441-445`) above 800 training rows -- at the sizes the
bench runs it (MI355X only).

* ``gp_love_kernel`` inside the solve's variance launch (all GPs of the step in one launch, points
  gathered from the stored previous solution) against ``oracle.love_var`` with the same Lanczos
  root: config 4 (quad2d, N=1000, H=30, B=1024: the thrust GP's root has rank ~12, the pitch GP's
  100, so the two widths share one launch) and config 5 (quad3d, N=4000, FITC mean on M=2000,
  H=40, variance at each GP's inputs, three rank-100 roots).  |var_gpu - var_oracle| <= 1e-9 sf2.
* config 5 at full size with the LOVE default against the C++ restatement using the same roots.

The LOVE restatement itself is parity unpinned (gpytorch is absent): tests/test_love_cpu.py pins its
algebra (R^T K R = I, LOVE variance within 0.1 % of the exact one, numpy = torch).
"""

from types import SimpleNamespace

import numpy as np
import pytest

from helpers import O, fitc_weights, initial_states, lqr, oracle_gps, problem, product_gps

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.parametrize("name,N,H,B,M", [("quad2d", 1000, 30, 1024, None), ("quad3d", 4000, 40, 128, 2000)])
def test_love_variance_kernel_matches_oracle_at_bench_sizes(name, N, H, B, M):
    torch = _torch()
    from gpmpc.solver import BatchSolver

    spec, data, hyp = problem(name, N)
    if name == "quad3d":
        spec.var_inputs = spec.gp_inputs          # bench config 5 (--var-inputs dynamics)
    gpp = product_gps(data, hyp)
    fitc = fitc_weights(gpp, M) if M else None
    gs = BatchSolver(spec, H, B)
    gs.set_gps(gpp, fitc=fitc, variance="love")   # the default: LOVE above 800 rows
    assert all(r is not None for r in gs.love_ranks), gs.love_ranks
    if name == "quad2d":   # 1-D thrust GP: Lanczos stops early -> two root widths in one launch
        assert gs.love_ranks[0] < 32 and gs.love_ranks[1] == 100, gs.love_ranks
    gs.set_tightening(True, 0.95, *lqr(spec))
    gs.reset(reset_iterate=True)
    x0, ph = initial_states(spec, spec.reference_trajectory(), B, seed=1)
    obs = torch.tensor(x0, device="cuda")
    ts = torch.tensor(ph, dtype=torch.int32, device="cuda")
    u = gs.solve(obs, ts)                          # first step: no previous solution, no variance
    assert (gs.status.cpu().numpy() == 0).all()
    xs, us, _ = (t.cpu().numpy() for t in gs.solution())
    gs.plant_step(obs, u, ts, out=obs)
    gs.solve(obs, ts)                              # variance launch at (xs, us)
    var = gs.variance().cpu().numpy()              # (B, H, n_gp)
    z = np.concatenate([xs[:, :-1, :], us], axis=2).reshape(B * H, -1)
    for g, (X, _) in enumerate(data):
        R = gpp[g].love_root(100).cpu().numpy()    # the root set_gps uploaded (seeded Lanczos)
        og = SimpleNamespace(X=X.reshape(N, -1), ell=hyp[g][0], sf2=hyp[g][1], sn2=hyp[g][2])
        ref = np.concatenate([O.love_var(og, R, z[c:c + 4096][:, spec.var_inputs[g]])
                              for c in range(0, B * H, 4096)])
        err = np.abs(var[:, :, g].reshape(-1) - ref).max()
        assert err <= 1e-9 * og.sf2, (g, err, og.sf2)


def test_config5_full_size_love_matches_cpp_restatement():
    """Config 5 as the bench runs it (LOVE tightening variance, FITC mean) against the C++
    restatement with the same roots, at KKT tolerance 1e-9."""
    torch = _torch()
    from oracle import cpu_ref
    from gpmpc.solver import BatchSolver

    if not cpu_ref.LIB_PATH.exists():
        pytest.skip("oracle/lib/libcpuref.so not built")
    spec, data, hyp = problem("quad3d", 4000)
    spec.var_inputs = spec.gp_inputs
    H, B, M, tol = 40, 4, 2000, 1e-9
    gpp = product_gps(data, hyp)
    fitc = fitc_weights(gpp, M)
    mats = lqr(spec)
    gs = BatchSolver(spec, H, B, tol=tol, qp_tol=1e-11, qp_max_iter=100)
    gs.set_var_inputs(spec.var_inputs)
    gs.set_gps(gpp, fitc=fitc, variance="love")
    gs.set_tightening(True, 0.95, *mats)
    gs.reset(reset_iterate=True)
    roots = [gp.love_root(100).cpu().numpy() for gp in gpp]
    ref = cpu_ref.CpuRef(spec, H, B, gps=oracle_gps(data, hyp), lqr_mats=mats, tol=tol, qp_tol=1e-11,
                         qp_max_iter=100, fitc=fitc, love_roots=roots)
    traj = spec.reference_trajectory()
    x0, ph = initial_states(spec, traj, B)
    plant = O.Dynamics(spec.to_dict(), None, params=spec.true_params)
    for k in range(3):
        gs.solve(torch.tensor(x0, device="cuda"), torch.tensor(ph + k, dtype=torch.int32, device="cuda"))
        u0 = ref.step(x0, ph + k, threads=4).copy()
        st = gs.status.cpu().numpy()
        np.testing.assert_array_equal(st, ref.status)
        assert (st == 0).all(), st
        xg, ug, tg = (t.cpu().numpy() for t in gs.solution())
        err = np.abs(xg - ref.x).max() / (1 + np.abs(ref.x).max())
        assert err <= 1e-6, (k, err)
        if k >= 1:
            assert tg[:, 1:, :].max() > 0.0
        for b in range(B):
            x0[b] = plant.rk4(x0[b], u0[b])[0]


@pytest.mark.parametrize("rank", [6, 40, 64, 100])
def test_love_kernel_tile_shapes(rank):
    """gp_love_kernel splits each root into full 16-column tiles and at most two 4-column quads on
    the 4-block MFMA (love_tiles): rank 6 (no full tile), 40 (two quads), 64 (tiles only), 100
    (six tiles and one quad), each against oracle.love_var with the uploaded root."""
    torch = _torch()
    from gpmpc.solver import BatchSolver

    spec, data, hyp = problem("quad2d", 400)
    gpp = product_gps(data, hyp)
    H, B = 30, 64
    gs = BatchSolver(spec, H, B)
    gs.set_gps(gpp, variance="love", love_rank=rank, love_force=True)
    gs.set_tightening(True, 0.95, *lqr(spec))
    gs.reset(reset_iterate=True)
    x0, ph = initial_states(spec, spec.reference_trajectory(), B, seed=3)
    obs = torch.tensor(x0, device="cuda")
    ts = torch.tensor(ph, dtype=torch.int32, device="cuda")
    u = gs.solve(obs, ts)
    xs, us, _ = (t.cpu().numpy() for t in gs.solution())
    gs.plant_step(obs, u, ts, out=obs)
    gs.solve(obs, ts)
    var = gs.variance().cpu().numpy()
    z = np.concatenate([xs[:, :-1, :], us], axis=2).reshape(B * H, -1)
    for g, (X, _) in enumerate(data):
        R = gs.love_roots[g]
        assert R is not None and R.shape[1] <= rank
        og = SimpleNamespace(X=X.reshape(400, -1), ell=hyp[g][0], sf2=hyp[g][1], sn2=hyp[g][2])
        ref = O.love_var(og, R, z[:, spec.var_inputs[g]])
        err = np.abs(var[:, :, g].reshape(-1) - ref).max()
        assert err <= 1e-9 * og.sf2, (rank, g, R.shape, err)
