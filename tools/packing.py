"""How well a multi-round SQP launch packs its instances onto the CUs (config 5: 512 quad3d instances,
one per CU, two rounds of workgroups), step by step over the driver's window.

Runs the closed loop the bench runs (same instances, initial states, phases, solver options, sequential
step: --overlap 0) and after every timed step reads each instance's solve time inside the SQP kernel
(stats slot 11, s_memrealtime ticks of that step) and the cost the kernel stored for the next dispatch
order (the SQP / IPM iteration counts of that step, StateDev::cost).  For each step it then schedules the
measured instance times greedily on `slots` CUs (a workgroup starts on the first CU to free up, in
dispatch order), for three orders:
  ranked   - by the previous step's cost, what the kernel dispatched (GPMPC_TUNE_ORDER 1)
  prevtime - by the previous step's measured solve times instead (a candidate predictor)
  ideal    - by this step's own times (longest first: what a perfect cost prediction would give)
  instance - instance order (GPMPC_TUNE_ORDER 0)
  xcd      - the ranked order with each workgroup bound to XCD (dispatch index % 8), 32 CUs each
and prints them beside the step's measured SQP-kernel time and the lower bound max(slowest instance,
sum of times / slots).  The schedule ignores contention between CUs, so "ranked" against the measured
time says how much of the kernel is packing and how much is the instances themselves.

  python3 tools/packing.py [--model quad3d --n-train 4000 --fitc 2000 --horizon 40 --batch 512 ...]
"""

import argparse
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gp-mpc_amd"))


def makespan(times, order, slots, xcds=1):
    """Greedy list schedule of `order` on `slots` CUs.  xcds > 1: the CUs split evenly over that many
    XCDs and the workgroup of dispatch index r goes to XCD r % xcds (each XCD then schedules its own
    subsequence on its own CUs), as the MI355X's command processor distributes workgroups."""
    end = 0.0
    for x in range(xcds):
        free = [0.0] * (slots // xcds)
        heapq.heapify(free)
        for b in list(order)[x::xcds]:
            t = heapq.heappop(free) + times[b]
            end = max(end, t)
            heapq.heappush(free, t)
    return end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="quad3d")
    ap.add_argument("--n-train", type=int, default=4000)
    ap.add_argument("--fitc", type=int, default=2000)
    ap.add_argument("--horizon", type=int, default=40)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--var-inputs", choices=["reference", "dynamics"], default="dynamics")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--slots", type=int, default=0, help="workgroups resident at once (0: one per CU)")
    ap.add_argument("--tail-work", type=float, default=0.0,
                    help="ms of extra work appended to every instance but the K last finishers: prints how far "
                         "it would extend the step's slowest instance for K = B/8, B/4, B/2 (0: skip)")
    args = ap.parse_args()

    import torch

    from gpmpc.gp import GaussianProcess
    from gpmpc.gpmpc import GPMPC
    from gpmpc.models import get_spec
    from gpmpc.solver import BatchSolver, setup_prior_dynamics
    from gpmpc.synthetic import DEFAULT_HYPERS, initial_states, make_training_data

    dev = torch.device("cuda", 0)
    spec = get_spec(args.model)
    if args.var_inputs == "dynamics":
        spec.var_inputs = spec.gp_inputs
    H, N, B = args.horizon, args.n_train, args.batch
    gps = []
    for i, (X, y) in enumerate(make_training_data(spec, N, seed=1)):
        gp = GaussianProcess(torch.tensor(X), torch.tensor(y))   # (as bench.py builds them)
        gp.set_hyperparameters(*DEFAULT_HYPERS[spec.name][i])
        gps.append(gp)
    fitc = None
    if args.fitc:
        for gp in gps:
            gp.K, gp.K_inv = gp.compute_covariances()
        me = type("Me", (), {})()
        me.gaussian_process, me.np_random = gps, np.random.default_rng(1337)
        fitc = GPMPC.precompute_sparse_posterior_mean(me, min(args.fitc, N))
    dfdx, dfdu = spec.prior_jacobian(np.zeros(spec.nx), spec.u_eq)
    lqr = setup_prior_dynamics(dfdx, dfdu, np.diag(spec.q_diag), np.diag(spec.r_diag), spec.dt)
    solver = BatchSolver(spec, H, B, device=dev)
    solver.set_tuning(overlap=0)
    solver.set_gps(gps, fitc=fitc, variance="love")   # bench.py's default
    solver.set_tightening(True, 0.95, *lqr)
    solver.reset(reset_iterate=True)
    x0, ph = initial_states(spec, spec.reference_trajectory(), B, seed=1)
    obs = torch.tensor(x0, device=dev)
    ts = torch.tensor(ph, dtype=torch.int32, device=dev)
    stats = torch.zeros(B, BatchSolver.STATS_SLOTS, dtype=torch.int64, device=dev)
    solver.set_stats(stats)
    slots = args.slots or torch.cuda.get_device_properties(0).multi_processor_count
    k_lin = 5 if spec.name == "quad3d" else 3   # SqpKernel::kCostLin (NB + 1 > 16 for quad3d)
    solver.set_profiling(True)
    prev_cost = prev_times = None
    rows = []
    for s in range(args.warmup + args.steps):
        before = stats[:, :2].clone()
        u = solver.solve(obs, ts)
        solver.plant_step(obs, u, ts, out=obs)
        torch.cuda.synchronize(dev)
        d = (stats[:, :2] - before).cpu().numpy()
        times = stats[:, 11].cpu().numpy() * 1e-5   # 100 MHz ticks -> ms
        cost = k_lin * d[:, 0] + 2 * d[:, 1]
        sqp_ms = solver.kernel_time_list()["sqp_ms"]
        if s >= args.warmup and prev_cost is not None:
            ranked = np.lexsort((np.arange(B), -prev_cost))   # order_by_cost_kernel: cost desc, index asc
            ideal = np.argsort(-times, kind="stable")
            prevt = np.argsort(-prev_times, kind="stable")
            rows.append({"step": s, "kernel_ms": sqp_ms[-1] if sqp_ms else None,
                         "ranked_ms": makespan(times, ranked, slots), "prevtime_ms": makespan(times, prevt, slots),
                         "ideal_ms": makespan(times, ideal, slots),
                         "instance_ms": makespan(times, np.arange(B), slots),
                         "xcd_ms": makespan(times, ranked, slots, 8),
                         "bound_ms": max(times.max(), times.sum() / slots), "slowest_ms": float(times.max()),
                         "mean_ms": float(times.mean()),
                         "p50_ms": float(np.percentile(times, 50)), "p75_ms": float(np.percentile(times, 75)),
                         "p90_ms": float(np.percentile(times, 90))})
            if args.tail_work > 0:
                srt = np.sort(times)
                for frac in (8, 4, 2):
                    K = B // frac
                    rows[-1][f"ext_k{K}_ms"] = float(max(0.0, srt[B - K - 1] + args.tail_work - srt[-1]))
        prev_cost, prev_times = cost.astype(np.float64), times.copy()
    print("step  kernel  ranked  prevtime  ideal  instance  xcd  bound  slowest  mean   (ms; schedules of the "
          "measured instance times)")
    for r in rows:
        print(f"{r['step']:4d}  {r['kernel_ms'] or float('nan'):6.3f}  {r['ranked_ms']:6.3f}  {r['prevtime_ms']:8.3f}  "
              f"{r['ideal_ms']:5.3f}  "
              f"{r['instance_ms']:8.3f}  {r['xcd_ms']:5.3f}  {r['bound_ms']:5.3f}  {r['slowest_ms']:7.3f}  {r['mean_ms']:5.3f}")
    mean = {k: float(np.mean([r[k] for r in rows])) for k in rows[0] if k != "step"}
    print("mean  " + "  ".join(f"{k} {v:.3f}" for k, v in mean.items()))
    print(json.dumps({"config": vars(args), "slots": slots, "mean": mean, "steps": rows}))


if __name__ == "__main__":
    main()
