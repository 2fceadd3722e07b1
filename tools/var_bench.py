"""Micro-benchmark of the large-N GP posterior kernel (gp_post_kernel, configs 4/5): one GP,
P points, N training rows; HIP-event time per launch, FP64 TFLOP/s by the DESIGN §2.2 count
(N(N+1) + 2N per point for the variance, 2N for the mean), and a torch fp64 check on a slice.

  python tools/var_bench.py [N ...]      (GPU only)
"""

import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gp-mpc_amd"), str(ROOT)]
from gpmpc.gp import GaussianProcess  # noqa: E402

PEAK = 78.6


def main():
    ns = [int(a) for a in sys.argv[1:]] or [1000, 4000]
    dev = "cuda:0"
    g = torch.Generator().manual_seed(0)
    for N in ns:
        d, P = 3, 30720
        X = torch.rand(N, d, generator=g, dtype=torch.float64) * 2 - 1
        y = torch.sin(3 * X).sum(1)
        gp = GaussianProcess(X, y)
        gp.set_hyperparameters(0.7, 2.0, 1e-4)
        Z = (torch.rand(P, d, generator=g, dtype=torch.float64) * 2 - 1).to(dev)
        for _ in range(3):
            mean, var = gp.predict(Z)
        torch.cuda.synchronize()
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            mean, var = gp.predict(Z)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        flops = P * (N * (N + 1) + 4 * N)
        # fp64 check on a slice
        lay = gp.device_layout(Z.device)
        zs = Z[:2048]
        k = gp.kernel(zs.cpu(), X).to(dev)
        v_ref = gp.outputscale - ((lay["Linv"][:N, :N] @ k.T) ** 2).sum(0)
        m_ref = k @ lay["alpha"].reshape(-1)
        err_v = ((var[:2048] - v_ref).abs() / v_ref.abs().clamp_min(1e-12)).max().item()
        err_m = ((mean[:2048] - m_ref).abs().max() / m_ref.abs().max()).item()
        tf = flops / ms * 1e-9
        print(f"N={N} P={P}: {ms:.3f} ms/launch, {tf:.1f} TFLOP/s = {100 * tf / PEAK:.1f} % of FP64 peak; "
              f"max rel err var {err_v:.2e} mean {err_m:.2e}", flush=True)


if __name__ == "__main__":
    main()
