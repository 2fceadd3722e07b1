#!/usr/bin/env python3
"""GP-MPC control steps/sec on MI355X (BASELINE.json metric, config 3 per GPU).

Workload (BASELINE.json metric): 2D quadrotor GP-MPC, N=200 GP training points, H=30, a global
batch of B=1024 independent MPC instances, split over the N GPUs in contiguous slices (strong
scaling, the metric's "batch 1024 @1/2/4/8 GPU"; ``--batch B`` instead fixes B instances per GPU:
weak scaling).  One "step" = one batched ``select_action`` over the B
instances (variance kernel -> tightening + SQP-GN/IPM kernel) followed by the synthetic
plant kernel that produces the next observation.  Inputs are resident in HBM; the GP,
hyperparameters, initial states and reference are synthetic and seeded
(gpmpc/synthetic.py).  N>1: one process per GPU (torch.distributed, RCCL), instances
sharded by rank, no collective in the data path; barrier + max-over-ranks timing.  With N>1 and
the default partition the line also carries ``weak_per_gpu``: the same step with 1024 instances on
every GPU (a second timed run, after the strong one).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

``--gpus N`` without torchrun launches the N ranks itself (gpmpc/launch.py, before any GPU
call).  ``--dry-run`` replaces the GPU step by a rank-dependent host sleep: it exercises the
launcher, the instance shards and the max-over-ranks timing on the CPU (gloo), for tests.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "gp-mpc_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

from gpmpc.launch import maybe_spawn, rank_env  # noqa: E402  (no GPU/torch.cuda use)

METRIC = "GP-MPC control steps/sec, 2D quadrotor H=30 N=200, batch 1024 @1/2/4/8 GPU"
METRIC_GLOBAL_BATCH = 1024   # the metric's batch, split over the GPUs (strong scaling)
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 dense peak (vector and matrix are equal on gfx950)
# exp_rbf (csrc/gpmpc_common.h) is 15 f64 VALU operations + 2 integer ones: the VALU ceiling of
# exps is the FP64 FMA-lane rate (78.6 TFLOP/s / 2) over 17 issued instructions
EXP_VALU_OPS = 17
EXP_CEILING_PER_S = FP64_PEAK_TFLOPS * 1e12 / 2 / EXP_VALU_OPS


def gp_flops(spec, n_train, H, love_ranks=None):
    """Algorithmic GP flops per instance.

    mean+gradient: per linearisation, per stage, per evaluation, per training point:
    2d (distance) + 2(d+1) (value + gradient contraction); state-dependent GPs are evaluated
    at the 4 RK4 points, u-only GPs once per stage.  variance: triangular L^-1 k (N(N+1))
    + squared norm (2N) per stage and GP.  exps counted separately.
    """
    per_lin = 0
    exps_lin = 0
    var = 0
    for g, d in enumerate(spec.gp_dims):
        state_dep = any(j < spec.nx for j in spec.gp_inputs[g])
        evals = 4 if state_dep else 1
        per_lin += H * evals * n_train * (4 * d + 2)
        exps_lin += H * evals * n_train
        r = love_ranks[g] if love_ranks else None
        # exact: triangular L^-1 k + squared norm; LOVE: R^T k (N x r) + squared norm
        var += H * (n_train * (n_train + 1) + 2 * n_train) if r is None else H * (2 * n_train * r + 2 * r)
    return per_lin, exps_lin, var


def love_tiles(rank):
    """gp_love_kernel's split of a rank-r root (gp_kernels.hip love_tiles): full 16-column tiles and
    at most two 4-column quads."""
    nf, rem = rank // 16, rank % 16
    nq = (rem + 3) // 4
    return (nf + 1, 0) if nq > 2 else (nf, nq)


def survey_flops_per_lin(spec, n_train, H):
    """SURVEY.md §8(d)'s per-linearisation count as written there: every GP at the 4 RK4 points
    (the reference's CasADi graph evaluates u-only GPs at each of them too)."""
    return sum(H * 4 * n_train * (4 * d + 2) for d in spec.gp_dims)


def cpu_threads() -> int:
    """Host cores this process may use (the GPU box exports OMP_NUM_THREADS = its CPU share)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_baseline(spec, data, hyp, H, seconds, lqr_mats, x0_all, phase_all, ids, warmup, steps, fitc=None,
                 love_roots=None, qp_tol=None):
    """Time the C++ CPU restatement (oracle/cpu_ref.cpp: SQP-GN + Mehrotra IPM with Riccati
    Newton steps, OpenMP over instances, the same tightening variance as the GPU leg: exact or
    the same LOVE roots) on the GPU leg's own window: the same global instance ids (an evenly
    spaced sample of them when the whole shard does not fit the CPU budget), the same initial
    states and reference phases, closed-loop steps 0 .. warmup-1 untimed and steps
    warmup .. warmup+steps-1 timed, as the GPU leg (the first, cold step is never timed,
    gpmpc/plotting.py:25).  All host cores over the sample (value), and a sub-sample with one
    instance at a time on one core (the reference's usage pattern)."""
    from oracle import cpu_ref
    from oracle import gpmpc_oracle as O

    gps = [O.ExactGP(X, y, *hyp[i]) for i, (X, y) in enumerate(data)]
    plant = O.Dynamics(spec.to_dict(), None, params=spec.true_params)
    ids = np.asarray(ids)
    threads = cpu_threads()
    window = warmup + steps

    def run(sel, nthreads):
        ref = cpu_ref.CpuRef(spec, H, len(sel), gps=gps, lqr_mats=lqr_mats, fitc=fitc, love_roots=love_roots,
                             qp_tol=qp_tol)
        x0 = x0_all[sel].copy()
        phase = phase_all[sel].astype(np.int32)
        elapsed, sqp = 0.0, 0
        for k in range(window):
            t0 = time.perf_counter()
            u0 = ref.step(x0, phase + k, threads=nthreads)
            dt = time.perf_counter() - t0
            if k >= warmup:
                elapsed += dt
                sqp += int(ref.sqp_iter.sum())
            for b in range(len(sel)):
                x0[b] = plant.rk4(x0[b], u0[b])[0]
        return elapsed, sqp

    # per-instance-step cost from one cold step of `threads` instances (an upper bound: the cold
    # step needs the most SQP iterations), then the largest sample the budget allows
    probe = ids[np.linspace(0, len(ids) - 1, min(threads, len(ids))).astype(int)]
    ref = cpu_ref.CpuRef(spec, H, len(probe), gps=gps, lqr_mats=lqr_mats, fitc=fitc, love_roots=love_roots,
                         qp_tol=qp_tol)
    t0 = time.perf_counter()
    ref.step(x0_all[probe].copy(), phase_all[probe].astype(np.int32), threads=threads)
    t_inst = (time.perf_counter() - t0) * threads / len(probe)     # core-seconds per instance-step
    n_all = int(0.65 * seconds * threads / (window * t_inst))
    n_all = max(min(threads, len(ids)), min(len(ids), n_all // threads * threads if n_all >= threads else n_all))
    sel = ids[np.linspace(0, len(ids) - 1, n_all).astype(int)] if n_all < len(ids) else ids
    el_all, sqp_all = run(sel, threads)
    n_one = max(1, min(len(sel), 64, int(0.35 * seconds / (window * t_inst))))
    sel1 = sel[np.linspace(0, len(sel) - 1, n_one).astype(int)]
    el_one, _ = run(sel1, 1)
    var = ("LOVE roots of ranks " + "/".join(str(None if R is None else R.shape[1]) for R in love_roots)
           if love_roots is not None and any(R is not None for R in love_roots) else "exact variance")
    return {"value": float(len(sel) * steps / el_all), "unit": "control steps/s", "cores": threads, "kind": "port",
            "single_instance_1core": float(len(sel1) * steps / el_one),
            "sqp_iter_mean": sqp_all / (len(sel) * steps),
            "instances": int(len(sel)), "window": [int(warmup), int(warmup + steps)],
            "sample": f"C++ restatement (oracle/cpu_ref.cpp, -O3 AVX2, OpenMP), {spec.name} N={data[0][0].shape[0]}"
                      f"{' FITC M=%d' % len(fitc[0][1]) if fitc else ''} H={H}, {var}: {len(sel)} of the GPU leg's "
                      f"{len(ids)} instances (same ids, initial states and reference phases), closed-loop steps "
                      f"{warmup}..{warmup + steps - 1} timed after {warmup} untimed, on {threads} threads; "
                      f"single_instance_1core: {len(sel1)} of them one at a time on 1 thread over the same steps"}


def single_instance_gpu(spec, gps, H, lqr_mats, x0, phase, warmup, steps, dev, qp_tol=None, qp_mu0=1.0,
                        variance="love"):
    """The reference's own usage pattern on the MI355X: the drop-in ``GPMPC.select_action(obs)``
    (B = 1, numpy in / out, host synchronisation) once per control step, timed with perf_counter
    around each call (`scripts/run_gp_mpc.py:55-57`) over the GPU leg's window for one of its
    instances; the untimed warm-up steps include the first one (`gpmpc/plotting.py:25`).  The
    environment step between calls (the synthetic plant kernel) is not timed.  HIP events on the
    same calls split the time into the variance and SQP kernels and the rest (host, launches,
    copies)."""
    import torch

    from gpmpc.gpmpc import GPMPC

    ctrl = GPMPC(spec, horizon=H, prob=0.95, batch=1, device=dev, variance=variance, qp_tol=qp_tol, qp_mu0=qp_mu0)
    ctrl.solver.set_tightening(True, 0.95, *lqr_mats)
    ctrl.set_gaussian_processes(gps)
    ctrl.reset()
    ctrl.traj_step = int(phase)
    obs = np.asarray(x0, dtype=np.float64).copy()
    times = []
    ctrl.solver.set_profiling(True)
    for k in range(warmup + steps):
        if k == warmup:
            ctrl.solver.kernel_time_list()   # keep the timed window's kernel events only
        t0 = time.perf_counter()
        u = ctrl.select_action(obs)
        dt = time.perf_counter() - t0
        if k >= warmup:
            times.append(dt)
        xt = torch.tensor(obs[None, :], device=dev)
        obs = ctrl.solver.plant_step(xt, torch.tensor(u[None, :], device=dev))[0].cpu().numpy()
    kt = ctrl.solver.kernel_time_list()
    ctrl.solver.set_profiling(False)
    t = np.array(times)
    sqp = float(np.mean(kt["sqp_ms"])) if kt["sqp_ms"] else None
    var = float(np.mean(kt["var_ms"])) if kt["var_ms"] else 0.0
    ms = float(t.mean() * 1e3)
    return {"value": float(len(t) / t.sum()), "unit": "control steps/s", "ms_per_step": ms,
            "p50_ms": float(np.median(t) * 1e3), "max_ms": float(t.max() * 1e3),
            "kernel_ms_per_step": {"sqp": sqp, "variance": var},
            "host_ms_per_step": None if sqp is None else ms - sqp - var,
            "sample": f"GPMPC.select_action(obs) at B=1 on the GPU (numpy in/out, host sync), one instance of the "
                      f"GPU leg (same initial state and reference phase), steps {warmup}..{warmup + steps - 1} "
                      f"timed with perf_counter after {warmup} untimed; host_ms = wall - kernel events"}


def _build_info():
    """Provenance of the library this run loaded (gpmpc_build_id against the tree's source hash)."""
    from gpmpc import _lib

    return _lib.build_info()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=None,
                    help="instances per GPU (weak scaling); default: the metric's global batch split over the GPUs")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="total instances over all GPUs, contiguous B/G slices per rank (strong scaling, "
                         f"SURVEY.md 8(e)); the default partition when --batch is not given ({METRIC_GLOBAL_BATCH})")
    ap.add_argument("--no-weak-secondary", action="store_true",
                    help="N>1, default partition: skip the second, weak-scaled run (weak_per_gpu)")
    ap.add_argument("--model", default="quad2d")
    ap.add_argument("--n-train", type=int, default=200)
    ap.add_argument("--horizon", type=int, default=30)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single-instance", action="store_true",
                    help="skip the B=1 drop-in timing (single_instance_gpu)")
    ap.add_argument("--qp-tol", type=float, default=None,
                    help="IPM tolerance of the QP sub-problems (default: the NLP tolerance 1e-6, as acados passes its "
                         "NLP tolerances on to the QP solver)")
    ap.add_argument("--qp-mu0", type=float, default=1.0)
    ap.add_argument("--seg", type=int, choices=[0, 1], default=None,
                    help="segment-parallel Newton solves on launches with two or four waves per instance "
                         "(gpmpc_set_tuning GPMPC_TUNE_SEG; default: the library's)")
    ap.add_argument("--overlap", type=int, choices=[0, 1], default=None,
                    help="overlapped halves for steps needing more than one round of workgroups "
                         "(gpmpc_set_tuning GPMPC_TUNE_OVERLAP; default: the library's)")
    ap.add_argument("--lin-cache", type=int, choices=[0, 1], default=None,
                    help="linearisation cache (gpmpc_set_tuning GPMPC_TUNE_LIN_CACHE; default: the library's)")
    ap.add_argument("--order", type=int, choices=[0, 1, 2], default=None,
                    help="cost-ordered dispatch (gpmpc_set_tuning GPMPC_TUNE_ORDER; default: the library's)")
    ap.add_argument("--var-split", type=int, choices=[0, 1, 4], default=None,
                    help="triangular variance kernel's column split (gpmpc_set_tuning GPMPC_TUNE_VAR_SPLIT)")
    ap.add_argument("--tail", type=int, default=None,
                    help="tail boost: the K costliest instances of a one-wave, one-round step as two-wave segment "
                         "solves beside the others' one-wave launch (gpmpc_set_tuning GPMPC_TUNE_TAIL: -1 as many as "
                         "the launch leaves SIMDs free, 0 off; default: the library's, -1)")
    ap.add_argument("--waves", type=int, choices=[0, 1, 2, 4], default=None,
                    help="SQP-kernel waves per instance (gpmpc_set_launch; default 0 = automatic)")
    ap.add_argument("--var-inputs", choices=["reference", "dynamics"], default="reference",
                    help="tightening-variance input map: the reference's (gpmpc.py:437-444) or each GP's own")
    ap.add_argument("--fitc", type=int, default=0, help="FITC mean on M inducing rows (config 5); 0 = exact GP")
    ap.add_argument("--variance", choices=["exact", "love"], default="love",
                    help="tightening variance: 'love' = the reference's gpytorch fast_pred_var (exact Cholesky up "
                         "to 800 training rows, rank-100 Lanczos root above; configs 2-3 are exact either way), "
                         "'exact' = L^-1 k at every size")
    ap.add_argument("--pmc-summary", default=str(ROOT / "profiles" / "pmc_current.json"),
                    help="tools/pmc_summary.py output of the same command (roofline.traffic)")
    ap.add_argument("--shard", default="",
                    help="R/N: run only rank R's slice of the N-rank partition, in this one process on one GPU "
                         "(measures one rank of a strong-scaled job; the job time is the max over its N shards, "
                         "tools/shard_sweep.sh); value then counts this shard's instances")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal: host sleep instead of the GPU step (launcher / shards / timing)")
    return ap.parse_args(argv)


def resolve_partition(args) -> bool:
    """Fix the instance partition: ``--global-batch G`` or, without ``--batch``, the metric's global
    batch (strong scaling); ``--batch B`` alone: B per GPU (weak).  Returns True when the weak
    secondary run applies (the default partition, so the line can show both figures)."""
    default = not args.global_batch and args.batch is None
    if default:
        args.global_batch = METRIC_GLOBAL_BATCH
    if args.global_batch:
        args.batch = None
    return default and not args.no_weak_secondary


def workload_name(spec, args, world=1):
    N, H, B = args.n_train, args.horizon, args.batch
    per = f"{B} instances per GPU" if not args.global_batch else f"global batch {args.global_batch} over {world} GPU(s)"
    return (f"{spec.name} GP-MPC N={N}{' FITC M=%d' % min(args.fitc, N) if args.fitc else ''} H={H}"
            f"{', variance at the GP inputs' if args.var_inputs == 'dynamics' else ''}"
            f"{', LOVE variance' if getattr(args, 'variance', 'exact') == 'love' and N > 800 else ''}"
            f"{', exact variance' if getattr(args, 'variance', 'exact') == 'exact' and N > 800 else ''}, "
            f"{per}, closed loop")


def init_dist(world, gpu, use_gpu):
    """torch.distributed process group (RCCL by default, GPMPC_DIST_BACKEND=gloo to rehearse)."""
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist

    backend = os.environ.get("GPMPC_DIST_BACKEND", "nccl" if use_gpu else "gloo")   # nccl = RCCL on ROCm
    if backend == "nccl":
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", gpu))
    else:
        dist.init_process_group(backend=backend)
    return dist


def reduce_timing(dist, elapsed, extra, dev=None):
    """Max over ranks of [elapsed, *extra] (the slowest rank sets the job's time)."""
    import torch

    t = torch.tensor([elapsed, *extra], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


WEAK_BATCH = 1024   # weak_per_gpu: instances per GPU of the secondary run (config 3's per-GPU batch)


def run_dry(args, rank, world, weak_secondary=False):
    """CPU rehearsal of the multi-rank bench: the same shards, barriers and max-over-ranks
    timing around a host sleep of (1 + rank) ms per step."""
    from gpmpc import distributed as D
    from gpmpc.models import get_spec

    dist = init_dist(world, 0, use_gpu=False)
    spec = get_spec(args.model)

    def timed(ids):
        for _ in range(args.warmup):
            time.sleep(1e-3 * (1 + rank))
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            time.sleep(1e-3 * (1 + rank))
        local = time.perf_counter() - t0   # this rank's own work, before the closing barrier
        if dist is not None:
            dist.barrier()
        elapsed, = reduce_timing(dist, time.perf_counter() - t0, [])
        shards = [None] * world
        if dist is not None:
            dist.all_gather_object(shards, [ids.start, ids.stop, local])
        else:
            shards = [[ids.start, ids.stop, local]]
        return elapsed, shards

    ids = D.shard_slice(args.global_batch, rank, world) if args.global_batch else D.shard_range(args.batch, rank)
    elapsed, shards = timed(ids)
    weak = None
    if weak_secondary and world > 1:
        w_el, w_shards = timed(D.shard_range(WEAK_BATCH, rank))
        weak = {"value": WEAK_BATCH * world * args.steps / w_el, "batch_per_gpu": WEAK_BATCH,
                "ms_per_step": w_el / args.steps * 1e3, "scaling": "weak", "shards": w_shards}
    if rank == 0:
        total = args.global_batch or args.batch * world
        print(json.dumps({"metric": METRIC, "value": total * args.steps / elapsed, "unit": "control steps/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
                          "scaling": "strong" if args.global_batch else "weak",
                          "vs_baseline": None, "dtype": "f64", "data": "dry run (host sleep, no GPU)",
                          "config": {"workload": workload_name(spec, args, world), "model": spec.name,
                                     "global_batch": total, "batch_per_gpu": len(ids), "horizon": args.horizon,
                                     "n_train": args.n_train, "parallelism": f"instances sharded over {world} rank(s)"},
                          "shards": shards, "weak_per_gpu": weak}))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def run_gpu(args, rank, local_rank, world, weak_secondary=False):
    import torch

    # one rank per GPU (local_rank modulo the visible GPUs only matters for a rehearsal of the
    # multi-rank path on fewer GPUs, with GPMPC_DIST_BACKEND=gloo)
    gpu = local_rank % max(torch.cuda.device_count(), 1)
    emulated = bool(args.shard)   # one rank of an N-rank job, alone (no process group)
    dist = None if emulated else init_dist(world, gpu, use_gpu=True)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)

    from gpmpc import distributed as D
    from gpmpc.gp import GaussianProcess
    from gpmpc.models import get_spec
    from gpmpc.solver import BatchSolver, setup_prior_dynamics
    from gpmpc.synthetic import DEFAULT_HYPERS, initial_states, make_training_data

    spec = get_spec(args.model)
    if args.var_inputs == "dynamics":
        spec.var_inputs = spec.gp_inputs
    H, N = args.horizon, args.n_train
    data = D.replicate_training_data(make_training_data(spec, N, seed=1), device=dev)  # GP replicated on every rank
    hyp = DEFAULT_HYPERS[spec.name]
    gps = []
    for i, (X, y) in enumerate(data):
        gp = GaussianProcess(torch.tensor(X), torch.tensor(y))
        gp.set_hyperparameters(*hyp[i])
        gps.append(gp)
    Q, R = np.diag(spec.q_diag), np.diag(spec.r_diag)
    dfdx, dfdu = spec.prior_jacobian(np.zeros(spec.nx), spec.u_eq)
    lqr_mats = setup_prior_dynamics(dfdx, dfdu, Q, R, spec.dt)
    fitc = None
    if args.fitc:
        from gpmpc.gpmpc import GPMPC

        for gp in gps:
            gp.K, gp.K_inv = gp.compute_covariances()
        me = type("Me", (), {})()
        me.gaussian_process, me.np_random = gps, np.random.default_rng(1337)
        fitc = GPMPC.precompute_sparse_posterior_mean(me, min(args.fitc, N))
    traj = spec.reference_trajectory()

    def measure(ids, total_instances):
        """One timed closed-loop run of this rank's instances ``ids`` (global ids of a
        ``total_instances`` job): W untimed steps, barrier + synchronize, K timed steps, barrier +
        synchronize, max over ranks."""
        B = len(ids)
        solver = BatchSolver(spec, H, B, device=dev, qp_tol=args.qp_tol, qp_mu0=args.qp_mu0)
        if args.seg is not None:
            solver.set_tuning(seg=args.seg)
        if args.overlap is not None:
            solver.set_tuning(overlap=args.overlap)
        for opt in ("lin_cache", "order", "var_split", "tail"):
            if getattr(args, opt) is not None:
                solver.set_tuning(**{opt: getattr(args, opt)})
        if args.waves is not None:
            solver.set_launch(waves=args.waves)
        solver.set_gps(gps, fitc=fitc, variance=args.variance)
        solver.set_tightening(True, 0.95, *lqr_mats)
        solver.reset(reset_iterate=True)
        x0_all, phase_all = initial_states(spec, traj, total_instances, seed=1)
        obs = torch.tensor(x0_all[ids.start:ids.stop], device=dev)
        tstep = torch.tensor(phase_all[ids.start:ids.stop], dtype=torch.int32, device=dev)
        stats_buf = torch.zeros(B, BatchSolver.STATS_SLOTS, dtype=torch.int64, device=dev)   # filled by the SQP kernel
        solver.set_stats(stats_buf)

        def step():
            u0 = solver.solve(obs, tstep)
            solver.plant_step(obs, u0, tstep, out=obs)

        solver.set_profiling(True)   # warm-up runs the timed body exactly (events)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
        solver.kernel_time_list()  # drop warm-up events
        stats_buf.zero_()
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        t_enqueue = time.perf_counter() - t0
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        solver.set_profiling(False)
        kt = solver.kernel_time_list()
        sqp_list, var_list = kt["sqp_ms"], kt["var_ms"]
        elapsed, sqp_sum, var_sum = reduce_timing(dist, elapsed, [sum(sqp_list), sum(var_list)], dev)
        tot = stats_buf.sum(0).to(torch.float64)
        mx = stats_buf.max(0).values.to(torch.float64)
        sums, status_counts, maxes = torch.cat([tot[:2], tot[9:10]]), tot[2:7].clone(), mx[7:9].clone()
        # per-instance solve time inside the SQP kernel (s_memrealtime, 100 MHz ticks, slot 10 summed over
        # the timed steps): the slowest instance's and the mean, for the roofline's latency block
        inst = torch.stack([mx[10], tot[10]])
        if dist is not None:
            dist.all_reduce(sums, op=dist.ReduceOp.SUM)
            dist.all_reduce(status_counts, op=dist.ReduceOp.SUM)
            dist.all_reduce(maxes, op=dist.ReduceOp.MAX)
            dist.all_reduce(inst[:1], op=dist.ReduceOp.MAX)
            dist.all_reduce(inst[1:], op=dist.ReduceOp.SUM)
        # instance-steps the statistics cover: every rank's (all-reduced) or, for an emulated shard
        # (no process group), this shard's own
        n_is = (B if emulated else total_instances) * args.steps
        return {"B": B, "solver": solver, "elapsed": elapsed, "launch": solver.launch_info(), "t_enqueue": t_enqueue, "sqp_list": sqp_list,
                "var_list": var_list, "sqp_sum": sqp_sum, "var_sum": var_sum, "x0_all": x0_all,
                "phase_all": phase_all, "value": total_instances * args.steps / elapsed,
                "sqp_mean": float(sums[0]) / n_is, "lin_mean": float(sums[2]) / n_is, "qp_mean": float(sums[1]) / n_is,
                "status_counts": status_counts, "maxes": maxes,
                "inst_ms_max": float(inst[0]) * 1e-5 / args.steps,                       # slowest instance
                "inst_ms_mean": float(inst[1]) * 1e-5 / args.steps / (B if emulated else total_instances)}

    # instances of this rank: contiguous global ids (strong: the rank's slice of the global batch;
    # weak: rank*B .. rank*B+B-1), no collective in the data path
    ids = D.shard_slice(args.global_batch, rank, world) if args.global_batch else D.shard_range(args.batch, rank)
    total_instances = args.global_batch or args.batch * world
    m = measure(ids, total_instances)
    if emulated:   # this shard's own throughput (the job's is the slowest shard's time over all of them)
        m["value"] = len(ids) * args.steps / m["elapsed"]
    weak = None
    if weak_secondary and world > 1 and not emulated:
        w = measure(D.shard_range(WEAK_BATCH, rank), WEAK_BATCH * world)
        weak = {"value": w["value"], "batch_per_gpu": WEAK_BATCH, "global_batch": WEAK_BATCH * world,
                "ms_per_step": w["elapsed"] / args.steps * 1e3, "scaling": "weak",
                "sqp_kernel_ms": w["sqp_sum"] / max(len(w["sqp_list"]), 1),
                "status_counts": {str(i): int(w["status_counts"][i]) for i in range(5)},
                "note": "secondary run: the same step with 1024 instances on every GPU (per-GPU work fixed)"}
    B, solver, elapsed = m["B"], m["solver"], m["elapsed"]
    sqp_list, var_list = m["sqp_list"], m["var_list"]
    sqp_mean, lin_mean, qp_mean = m["sqp_mean"], m["lin_mean"], m["qp_mean"]
    status_counts, maxes = m["status_counts"], m["maxes"]

    if rank == 0 or emulated:   # an emulated shard is the only process: it always reports
        # a step run as overlapped halves (gpmpc_get_launch_info): the events bracket spans of the step
        # (the costlier half's variance launch; then both SQP launches plus the cheaper half's
        # variance launch), not kernel durations -- no per-kernel figure is derived from them
        overlapped = m["launch"]["overlapped"]
        per_lin, exps_lin, var_flops = gp_flops(spec, N, H, getattr(solver, "love_ranks", None))
        # dominant kernel: the SQP kernel; linearisations computed per instance-step = sqp_iter + 1,
        # minus the one read from the linearisation cache (lin_mean, counted by the kernel)
        sqp_ms = m["sqp_sum"] / max(len(sqp_list), 1)
        var_ms = m["var_sum"] / max(len(var_list), 1)
        # overlapped: the SQP flops over the step's whole kernel span (variance + SQP spans), a lower
        # bound on the SQP kernel's rate; the kernel's own duration comes from a rocprofv3 trace
        sqp_basis_ms = sqp_ms + (var_ms if var_list else 0.0) if overlapped else sqp_ms
        # SURVEY.md §8(d)'s count: F_mean = K_sqp H 4 sum_g N_g (4 d_g + 2) per instance-step with
        # K_sqp = sqp_iter_mean (every GP at the 4 RK4 points of every SQP iteration), per launch
        flops_8d = B * sqp_mean * survey_flops_per_lin(spec, N, H)
        achieved = flops_8d / (sqp_basis_ms * 1e-3) / 1e12
        # what the kernel executes: linearisations computed (slot 9: one per SQP iteration plus the
        # converged iterate's, minus the cached one), u-only GPs once per stage
        flops_exec = B * lin_mean * per_lin
        achieved_exec = flops_exec / (sqp_basis_ms * 1e-3) / 1e12
        var_tf = (B * var_flops) / (var_ms * 1e-3) / 1e12 if var_list and not overlapped else None
        exps_launch = B * lin_mean * exps_lin
        workload = workload_name(spec, args, world)
        traffic, traffic_src = None, None
        try:
            with open(args.pmc_summary) as fh:
                pmc = json.load(fh)
            if pmc.get("config", {}).get("workload") == workload:
                pre = "gpmpc::sqp_step_kernel<%d" % spec.model_id   # <ID> or <ID, split-layout flag>
                e = next((v for kname, v in pmc["kernels"].items() if kname.startswith(pre)), {})
                traffic = e.get("hbm_bytes_est")
                if traffic is not None:
                    traffic_src = (f"{os.path.relpath(args.pmc_summary, ROOT)} (rocprofv3 FETCH_SIZE / WRITE_SIZE passes "
                                   f"of this command, committed; 2 x FETCH + WRITE per launch)")
        except (OSError, ValueError, KeyError):
            traffic = None
        single = None
        if world == 1 and not emulated and not args.no_single_instance and not args.fitc:
            single = single_instance_gpu(spec, gps, H, lqr_mats, m["x0_all"][ids.start], m["phase_all"][ids.start],
                                         args.warmup, args.steps, dev, qp_tol=args.qp_tol, qp_mu0=args.qp_mu0,
                                         variance=args.variance)
        cpu = None
        if world == 1 and not args.no_cpu_baseline and not emulated:   # rank 0 at N=1 only
            cpu = cpu_baseline(spec, data, hyp, H, args.cpu_seconds, lqr_mats, m["x0_all"], m["phase_all"], list(ids),
                               args.warmup, args.steps, fitc=fitc, love_roots=solver.love_roots, qp_tol=args.qp_tol)
        sq = np.array(sqp_list) if sqp_list else np.zeros(1)
        out = {
            "metric": METRIC,
            "value": m["value"],
            "unit": "control steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.global_batch else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded GP training set, initial states, figure-eight reference)",
            "config": {"workload": workload,
                       "model": spec.name, "global_batch": total_instances, "horizon": H, "n_train": N,
                       "batch_per_gpu": B,
                       "parallelism": f"instances sharded over {world} GPU(s) in contiguous slices, GP replicated"},
            "roofline": {"kernel": "sqp_step_kernel", "bound": "mfma", "regime": "latency",
                         "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic, "traffic_source": traffic_src,
                         "flops_per_launch": flops_8d,
                         "count": "SURVEY.md 8(d): F_mean = K_sqp * H * 4 * sum_g N_g (2 d_g + 2 (d_g + 1)) per "
                                  "instance-step, K_sqp = sqp_iter_mean; x instances of the launch",
                         "note": "the FP64 MFMA peak is the ceiling the fraction is priced against (the GP sums are "
                                 "the kernel's one dense contraction); the kernel does not run at that ceiling: it "
                                 "is latency-bound, set by its slowest instance's sequential recursions (latency)",
                         "time_basis": ("overlapped step: SQP flops over the step's whole kernel span (variance + "
                                        "SQP event spans, a lower bound on the SQP kernel's rate)") if overlapped
                                       else "SQP-kernel HIP events",
                         "latency": {"slowest_instance_ms_per_step": m["inst_ms_max"],
                                     "mean_instance_ms_per_step": m["inst_ms_mean"],
                                     "kernel_ms_per_step": sqp_basis_ms,
                                     "slowest_over_kernel": m["inst_ms_max"] / sqp_basis_ms,
                                     "slowest_over_mean": m["inst_ms_max"] / max(m["inst_ms_mean"], 1e-12),
                                     "note": "each instance's time inside the SQP kernel (s_memrealtime, first to last "
                                             "instruction of its workgroup, stats slot 10) summed over the timed steps; "
                                             "slowest_over_kernel near 1: the launch lasts as long as its slowest "
                                             "instance's critical path"},
                         "executed": {"achieved": achieved_exec, "frac": achieved_exec / FP64_PEAK_TFLOPS,
                                      "flops_per_launch": flops_exec,
                                      "note": "flops the kernel executes: linearisations computed (the cached one "
                                              "skipped, the converged iterate's included), u-only GPs once per stage"}},
            "roofline_variance": None if var_tf is None else {
                "kernel": ((f"gp_love_kernel<true> (LOVE root ranks {'/'.join(str(r) for r in solver.love_ranks if r)}, "
                            f"full tiles/quads {'/'.join('%d+%d' % love_tiles(r) for r in solver.love_ranks if r)})")
                           if any(getattr(solver, "love_ranks", None) or [])
                           else (f"gp_var_tri_kernel<{(N + 15) // 16},true>" if (N + 15) // 16 <= 16
                                 else "gp_post_kernel<true,FULL>")),
                "bound": "mfma", "achieved": var_tf, "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": var_tf / FP64_PEAK_TFLOPS, "ms_per_launch": var_ms},
            "launch": {**m["launch"], "note": ("overlapped halves: kernel_ms_per_step and roofline_variance are null "
                                               "(the HIP events bracket spans of the step, not kernels); "
                                               "step_span_ms_per_step holds the spans; per-kernel durations come "
                                               "from rocprofv3 kernel traces") if overlapped else "one variance "
                                               "launch, then one SQP launch, each bracketed by HIP events"},
            "exp_ceiling": {"exps_per_launch": exps_launch, "achieved_per_s": exps_launch / (sqp_basis_ms * 1e-3),
                            "ceiling_per_s": EXP_CEILING_PER_S,
                            "frac": exps_launch / (sqp_basis_ms * 1e-3) / EXP_CEILING_PER_S,
                            "note": f"GP-phase exps over the whole SQP-kernel time; ceiling = FP64 VALU FMA-lane "
                                    f"rate / {EXP_VALU_OPS} instructions per exp_rbf"},
            "kernel_ms_per_step": None if overlapped else {"sqp": sqp_ms, "variance": var_ms},
            "step_span_ms_per_step": {"first_half_variance": var_ms, "sqp_and_second_half_variance": sqp_ms}
                                     if overlapped else None,
            "sqp_kernel_ms_per_step_distribution": {
                "min": float(sq.min()), "p50": float(np.median(sq)), "p90": float(np.percentile(sq, 90)),
                "max": float(sq.max()), "per_step": [round(float(v), 4) for v in sq],
                "basis": "SQP-and-second-half-variance span (overlapped step)" if overlapped else "SQP-kernel events"},
            "host_enqueue_ms_per_step": m["t_enqueue"] / args.steps * 1e3,
            "sqp_iter_mean": sqp_mean,
            "linearisations_per_step": lin_mean,
            "sqp_iter_max": int(maxes[0]),
            "qp_iter_mean_per_step": qp_mean,
            "qp_iter_max_per_step": int(maxes[1]),
            "status_counts": {str(i): int(status_counts[i]) for i in range(5)},
            "exps_per_sqp_launch": exps_launch,
            "weak_per_gpu": weak,
            "single_instance_gpu": single,
            "cpu_baseline": cpu,
            "build": _build_info(),
        }
        if emulated:
            out["emulated_shard"] = {"rank": rank, "world": world, "instances": [ids.start, ids.stop],
                                     "note": "one rank of the N-rank partition run alone on one GPU; value = this "
                                             "shard's instances x steps / its time"}
        print(json.dumps(out))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    # N ranks without torchrun: relaunch under torch.distributed.run before touching the GPU
    maybe_spawn(args.gpus, str(Path(__file__).resolve()), argv)
    rank, local_rank, world = rank_env()
    if args.shard:
        if world != 1 or args.dry_run:
            raise SystemExit("--shard R/N runs one rank alone: start it as a single process")
        rank, world = (int(v) for v in args.shard.split("/"))
        if not 0 <= rank < world:
            raise SystemExit("--shard R/N needs 0 <= R < N")
        args.gpus = world
    elif world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    weak_secondary = resolve_partition(args)
    if args.dry_run:
        run_dry(args, rank, world, weak_secondary)
    else:
        run_gpu(args, rank, local_rank, world, weak_secondary)


if __name__ == "__main__":
    main()
