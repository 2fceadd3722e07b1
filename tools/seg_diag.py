#!/usr/bin/env python3
"""Diagnostic: one closed-loop step of the segment-parallel solve against the one-wave recursion
(same instances), per launch shape; prints status / iteration counts / solution differences."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gp-mpc_amd"), str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import initial_states, lqr, problem, product_gps  # noqa: E402
from gpmpc.solver import BatchSolver  # noqa: E402

for name, N, H in (("cartpole", 200, 30), ("quad2d", 200, 30)):
    spec, data, hyp = problem(name, N)
    B = 4
    x0, ph = initial_states(spec, spec.reference_trajectory(), B)
    res = {}
    for waves, seg, mi in ((1, 0, 25), (2, 1, 25), (4, 1, 25)):
        s = BatchSolver(spec, H, B, tol=1e-9, qp_tol=1e-11, qp_max_iter=100, max_iter=mi)
        s.set_launch(waves=waves)
        s.set_tuning(seg=seg)
        s.set_gps(product_gps(data, hyp))
        s.set_tightening(True, 0.95, *lqr(spec))
        s.reset(reset_iterate=True)
        s.solve(torch.tensor(x0, device="cuda"), torch.tensor(ph, dtype=torch.int32, device="cuda"))
        x, u, _ = (t.cpu().numpy() for t in s.solution())
        res[(waves, seg, mi)] = (x, u)
        print(name, "waves", waves, "seg", seg, "max_iter", mi, "status", s.status.cpu().tolist(), "sqp", s.sqp_iter.cpu().tolist(),
              "qp", s.qp_iter.cpu().tolist(), "res", np.array2string(s.res.cpu().numpy().max(0), precision=2),
              "dx vs 1-wave", float(np.abs(x - res[(1, 0, 25)][0]).max()), "du", float(np.abs(u - res[(1, 0, 25)][1]).max()),
              flush=True)
