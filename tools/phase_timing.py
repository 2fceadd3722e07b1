#!/usr/bin/env python3
"""Phase breakdown of the SQP kernel with the diagnostic build (in-kernel s_memtime stamps).

    make -C gp-mpc_amd/csrc timing && python tools/phase_timing.py [--model quad2d --batch 1024]

Prints the mean shader-clock cycles per instance spent in each phase of one closed-loop
step (after warm-up), and the share of the step.  Diagnostic only: the stamps themselves
perturb the kernel; read the shares, not the absolute time.
"""

import argparse
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
os.environ.setdefault("GPMPC_LIB", str(ROOT / "gp-mpc_amd" / "gpmpc" / "lib" / "libgpmpc_mi355x_timing.so"))
sys.path.insert(0, str(ROOT / "gp-mpc_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

PHASES = ["tighten", "linearize", "resid/setup", "ipm-vector", "ric-factor", "ric-vector", "forward", "other",
          "acl-maps", "recover", "ipm-resid", "(gp-sums within linearize)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="quad2d")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--n-train", type=int, default=200)
    ap.add_argument("--horizon", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--no-gp", action="store_true", help="nominal dynamics (isolates the GP sums)")
    ap.add_argument("--fitc", type=int, default=0, help="FITC mean on M inducing rows (config 5)")
    ap.add_argument("--var-inputs", choices=["reference", "dynamics"], default="reference")
    ap.add_argument("--dump", default="", help="save the per-step per-instance phase cycles (.npy)")
    ap.add_argument("--waves", type=int, default=0, help="waves per instance (gpmpc_set_launch; 0 = auto)")
    ap.add_argument("--seg", type=int, default=None, help="two-segment Newton solves (gpmpc_set_tuning GPMPC_TUNE_SEG)")
    args = ap.parse_args()
    from gpmpc import _lib
    from gpmpc.gp import GaussianProcess
    from gpmpc.models import get_spec
    from gpmpc.solver import BatchSolver, setup_prior_dynamics
    from gpmpc.synthetic import DEFAULT_HYPERS, initial_states, make_training_data

    spec = get_spec(args.model)
    if args.var_inputs == "dynamics":
        spec.var_inputs = spec.gp_inputs
    H, B, N = args.horizon, args.batch, args.n_train
    data = make_training_data(spec, N, seed=1)
    gps = []
    for i, (X, y) in enumerate(data):
        gp = GaussianProcess(torch.tensor(X), torch.tensor(y))
        gp.set_hyperparameters(*DEFAULT_HYPERS[spec.name][i])
        gps.append(gp)
    dfdx, dfdu = spec.prior_jacobian(np.zeros(spec.nx), spec.u_eq)
    mats = setup_prior_dynamics(dfdx, dfdu, np.diag(spec.q_diag), np.diag(spec.r_diag), spec.dt)
    s = BatchSolver(spec, H, B)
    s.set_launch(waves=args.waves)
    if args.seg is not None:
        s.set_tuning(seg=args.seg)
    if args.no_gp:
        s.set_gps(None)
    else:
        fitc = None
        if args.fitc:
            from gpmpc.gpmpc import GPMPC

            for gp in gps:
                gp.K, gp.K_inv = gp.compute_covariances()
            me = type("Me", (), {})()
            me.gaussian_process, me.np_random = gps, np.random.default_rng(1337)
            fitc = GPMPC.precompute_sparse_posterior_mean(me, min(args.fitc, N))
        s.set_gps(gps, fitc=fitc)
        s.set_tightening(True, 0.95, *mats)
    s.reset(True)
    tbuf = torch.zeros(B, len(PHASES), dtype=torch.int64, device="cuda")
    _lib.check(s.lib.gpmpc_set_timing_buffer(s._h, tbuf.data_ptr()))
    traj = spec.reference_trajectory()
    x0, ph = initial_states(spec, traj, B)
    obs = torch.tensor(x0, device="cuda")
    ts = torch.tensor(ph, dtype=torch.int32, device="cuda")
    for _ in range(args.warmup):
        u0 = s.solve(obs, ts)
        s.plant_step(obs, u0, ts, out=obs)
    tot = np.zeros(len(PHASES))
    crit = np.zeros(len(PHASES))   # the slowest instance of each step (it sets the kernel time)
    per_step = []
    s.set_profiling(True)
    s.kernel_times()
    for _ in range(args.steps):
        u0 = s.solve(obs, ts)
        torch.cuda.synchronize()
        tb = tbuf.cpu().numpy().astype(np.float64)
        per_step.append(tb.copy())
        tot += tb.mean(0)
        crit += tb[np.argmax(tb[:, :-1].sum(1))]
        s.plant_step(obs, u0, ts, out=obs)
    kt = s.kernel_times()
    if args.dump:
        np.save(args.dump, np.stack(per_step))
    cyc = tot / args.steps
    sub = cyc[-1]            # GP sums: a sub-phase of "linearize", not part of the total
    cyc = cyc[:-1]
    ms = kt["sqp_ms"] / max(kt["sqp_launches"], 1)
    print(f"waves {args.waves or 'auto'}")
    print(f"{spec.name} B={B} H={H} N={N}: sqp kernel {ms:.3f} ms/launch, sqp_iter {s.sqp_iter.float().mean():.2f}, "
          f"qp_iter {s.qp_iter.float().mean():.2f}")
    print(f"cycles per instance (mean) {cyc.sum():.0f} -> {cyc.sum() / (ms * 1e-3) / 1e9:.2f} G cycles/s effective")
    crit /= args.steps
    csub, crit = crit[-1], crit[:-1]
    print(f"{'phase':26s} {'mean instance':>22s} {'slowest instance per step':>30s}")
    for name, c, k in zip(PHASES, cyc, crit):
        print(f"  {name:24s} {c:10.0f} cyc {100 * c / cyc.sum():5.1f} %   {k:10.0f} cyc {100 * k / crit.sum():5.1f} %")
    print(f"  {PHASES[-1]:24s} {sub:10.0f} cyc {100 * sub / cyc.sum():5.1f} %   {csub:10.0f} cyc {100 * csub / crit.sum():5.1f} %")
    print(f"  {'total':24s} {cyc.sum():10.0f} cyc           {crit.sum():10.0f} cyc")


if __name__ == "__main__":
    main()
