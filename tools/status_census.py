#!/usr/bin/env python3
"""Status census of the vs-C++ parity configurations at KKT tolerance 1e-9 (GPU only).

Runs the closed loops of tests/test_gpu_parity.py::test_closed_loop_parity_vs_cpp_restatement and
tests/test_gpu_launch.py on the GPU alone and prints, per configuration and step, the status
counts and the largest SQP iteration count, so the tests can assert "every instance converges"
exactly where that holds.  Output: one JSON line per configuration.
"""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gp-mpc_amd"), str(ROOT), str(ROOT / "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import initial_states, lqr, problem, product_gps  # noqa: E402
from gpmpc.solver import BatchSolver  # noqa: E402

CASES = [("quad3d", 100, 40, 8, 4, "dynamics", 0), ("quad3d", 100, 40, 8, 3, "reference", 0),
         ("quad2d", 200, 30, 16, 4, "reference", 0), ("cartpole", 50, 20, 16, 6, "reference", 0)]
for w in (1, 2, 4):
    CASES += [("quad2d", 200, 30, 12, 4, "reference", w), ("cartpole", 50, 20, 12, 4, "reference", w),
              ("quad2d", 120, 15, 6, 3, "reference", w), ("cartpole", 40, 10, 6, 3, "reference", w)]

for name, N, H, B, steps, var, waves in CASES:
    spec, data, hyp = problem(name, N)
    if var == "dynamics":
        spec.var_inputs = spec.gp_inputs
    gs = BatchSolver(spec, H, B, tol=1e-9, qp_tol=1e-11, qp_max_iter=100)
    if waves:
        gs.set_launch(waves=waves)
    gs.set_gps(product_gps(data, hyp))
    gs.set_tightening(True, 0.95, *lqr(spec))
    gs.reset(reset_iterate=True)
    x0, ph = initial_states(spec, spec.reference_trajectory(), B)
    obs = torch.tensor(x0, device="cuda")
    ts = torch.tensor(ph, dtype=torch.int32, device="cuda")
    rec = []
    for s in range(steps):
        u = gs.solve(obs, ts)
        st = gs.status.cpu().numpy()
        rec.append({"counts": np.bincount(st, minlength=5).tolist(), "sqp_max": int(gs.sqp_iter.max()),
                    "res_max": float(gs.res.max())})
        gs.plant_step(obs, u, ts, out=obs)
    print(json.dumps({"case": [name, N, H, B, steps, var, waves], "steps": rec}), flush=True)
