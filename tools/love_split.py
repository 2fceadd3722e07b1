#!/usr/bin/env python3
"""Where the LOVE variance kernel's time goes at config 4 (quad2d, N=1000, H=30, B=1024).

gp_love_kernel<NTC> runs every GP of the step in one launch (grid.y = GP); GP g's blocks do
N/4 K-steps of ceil(r_g / 16) MFMAs each (r_g: its root rank, 12 for the 1-D thrust GP and 100
for the pitch GP, padded to 16 and 112 columns) against the same N exps per point.  This script
times the variance launch (HIP events, the bench's own timer) with the pitch GP's root at rank
100 (7 column tiles, the default), 96 (6 tiles: the padding of the 7th tile removed) and 16
(1 tile), the thrust root unchanged, and reports the per-tile cost.

    python tools/love_split.py  (on the GPU box)
"""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gp-mpc_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gpmpc.gp import GaussianProcess  # noqa: E402
from gpmpc.models import get_spec  # noqa: E402
from gpmpc.solver import BatchSolver, setup_prior_dynamics  # noqa: E402
from gpmpc.synthetic import DEFAULT_HYPERS, initial_states, make_training_data  # noqa: E402


def run(pitch_rank, steps=20, warmup=5):
    spec = get_spec("quad2d")
    H, B, N = 30, 1024, 1000
    data = make_training_data(spec, N, seed=1)
    gps = []
    for i, (X, y) in enumerate(data):
        gp = GaussianProcess(torch.tensor(X), torch.tensor(y))
        gp.set_hyperparameters(*DEFAULT_HYPERS["quad2d"][i])
        gps.append(gp)
    Q, R = np.diag(spec.q_diag), np.diag(spec.r_diag)
    dfdx, dfdu = spec.prior_jacobian(np.zeros(spec.nx), spec.u_eq)
    s = BatchSolver(spec, H, B)
    s.set_gps(gps, variance="love")
    if pitch_rank != 100:   # replace the pitch GP's root by a rank-`pitch_rank` root
        Rp = gps[1].love_root(pitch_rank).cpu().numpy()
        Rp = np.ascontiguousarray(Rp)
        from gpmpc import _lib

        _lib.check(s.lib.gpmpc_set_gp_variance_root(s._h, 1, Rp.shape[0], Rp.shape[1], Rp.ctypes.data))
        s.love_ranks[1] = Rp.shape[1]
    s.set_tightening(True, 0.95, *setup_prior_dynamics(dfdx, dfdu, Q, R, spec.dt))
    s.reset(reset_iterate=True)
    x0, ph = initial_states(spec, spec.reference_trajectory(), B, seed=1)
    obs = torch.tensor(x0, device="cuda")
    ts = torch.tensor(ph, dtype=torch.int32, device="cuda")
    s.set_profiling(True)
    for k in range(warmup + steps):
        if k == warmup:
            torch.cuda.synchronize()
            s.kernel_time_list()
        u = s.solve(obs, ts)
        s.plant_step(obs, u, ts, out=obs)
    torch.cuda.synchronize()
    kt = s.kernel_time_list()
    return {"pitch_rank": pitch_rank, "roots": s.love_ranks, "var_ms": float(np.mean(kt["var_ms"])),
            "var_ms_min": float(np.min(kt["var_ms"]))}


if __name__ == "__main__":
    out = [run(r) for r in (100, 96, 16)]
    for o in out:
        print(json.dumps(o))
    full, r96, r16 = (o["var_ms_min"] for o in out)
    print(json.dumps({"per_pitch_tile_ms": (full - r16) / 6, "padding_tile_share_of_launch": (full - r96) / full,
                      "pitch_tiles_share_of_launch": (full - r16) / full}))
