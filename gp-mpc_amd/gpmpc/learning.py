"""Episodic GP-MPC learning loop on the MI355X (`scripts/run_gp_mpc.py:42-137`).

The reference runs one crazyflow environment on the CPU, collects transitions with the prior
MPC, fits the GPs, and re-runs with GP-MPC each epoch.  Here an "environment" is the batched
synthetic plant kernel (``BatchSolver.plant_step``: RK4 of the model with its true
parameters), so B episodes run at once on the GPU; transitions are gathered from all of them.

* :func:`run_evaluation` -- one closed-loop episode per instance (`run_gp_mpc.py:42-72`)
* :func:`sample_data`    -- random transitions of an episode batch (`run_gp_mpc.py:75-83`)
* :func:`learn`          -- prior run, then per epoch: sample, ``preprocess_data``,
  ``train_gp`` (on the GPU; data-parallel under torch.distributed), ``reset``, test and
  train episodes (`run_gp_mpc.py:86-137`).  Under N ranks every rank runs its own contiguous
  shard of the instances and the newly sampled transitions are all-gathered each epoch, so
  every rank fits the same GPs on the same data.
* :func:`get_runtime` / :func:`save_runtime_csv` -- the runtime summary and CSV of
  `gpmpc/plotting.py:10-62`.
"""

from __future__ import annotations

import time
from pathlib import Path

import numpy as np
import torch

from .synthetic import initial_states


def run_evaluation(ctrl, x0: np.ndarray, steps: int, tstep0: np.ndarray | None = None, plant_solver=None) -> dict:
    """Closed-loop episodes of ``steps`` control steps for B instances at once.

    ``ctrl`` is a :class:`~gpmpc.gpmpc.GPMPC` or :class:`~gpmpc.mpc.MPC` with ``batch = B``;
    the plant is the synthetic true-parameter model of the same spec.  Returns numpy arrays
    ``obs`` (steps+1, B, nx), ``action`` (steps, B, nu), ``status`` (steps, B),
    ``inference_time_data`` (steps,) seconds per batched select_action (synchronised).
    """
    ctrl.reset()
    solver = plant_solver if plant_solver is not None else ctrl.solver
    dev = solver.device
    B = solver.batch
    obs = torch.tensor(np.asarray(x0, dtype=np.float64).reshape(B, -1), device=dev)
    ts = torch.tensor(np.zeros(B) if tstep0 is None else tstep0, dtype=torch.int32, device=dev)
    data = {"obs": [obs.cpu().numpy()], "action": [], "status": [], "inference_time_data": []}
    for _ in range(steps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        u = ctrl.select_action_batch(obs, ts.clone())
        torch.cuda.synchronize(dev)
        data["inference_time_data"].append(time.perf_counter() - t0)
        data["action"].append(u.cpu().numpy())
        data["status"].append(ctrl.solver.status.cpu().numpy())
        obs = solver.plant_step(obs, u, ts)   # advances the reference index too
        data["obs"].append(obs.cpu().numpy())
    return {k: np.array(v) for k, v in data.items()}


def sample_data(data: dict, n_samples: int, rng: np.random.Generator):
    """Random transitions (x, u, x_next) from an episode batch (`scripts/run_gp_mpc.py:75-83`):
    the (step, instance) pairs are sampled without replacement."""
    steps, B = data["action"].shape[:2]
    n = steps * B
    idx = rng.choice(n, n_samples, replace=False) if n_samples < n else np.arange(n)
    k, b = idx // B, idx % B
    return data["obs"][k, b], data["action"][k, b], data["obs"][k + 1, b]


def tracking_cost(data: dict, traj: np.ndarray, tstep0: np.ndarray | None = None) -> float:
    """Mean squared position-state tracking error of an episode batch against the reference."""
    obs = data["obs"][1:]
    steps, B = obs.shape[:2]
    t0 = np.zeros(B, dtype=int) if tstep0 is None else np.asarray(tstep0, dtype=int)
    idx = (t0[None, :] + 1 + np.arange(steps)[:, None]) % traj.shape[1]
    ref = traj[:, idx].transpose(1, 2, 0)
    return float(((obs - ref) ** 2).sum(-1).mean())


def learn(n_epochs: int, ctrl, lr: float, gp_iterations: int, seed: int, samples_per_epoch: int,
          episode_len: int, x0: np.ndarray | None = None, tstep0: np.ndarray | None = None):
    """Episodic learning (`scripts/run_gp_mpc.py:86-137`): epoch 0 runs the prior MPC; every
    epoch then fits the GPs on all data gathered so far and runs a test and a train episode
    batch with GP-MPC.  Returns (train_runs, test_runs, timing) dicts keyed by epoch."""
    from . import distributed as D

    spec = ctrl.model
    rank, size = D.world()
    rng = np.random.default_rng(seed if size == 1 else [seed, rank])
    B = ctrl.batch
    if x0 is None:   # this rank's shard of the B * size instances
        ids = D.shard_range(B, rank)
        x0_all, t_all = initial_states(spec, ctrl.traj, B * size, seed=seed)
        x0, tstep0 = x0_all[ids.start:ids.stop], t_all[ids.start:ids.stop]
    train_runs, test_runs, timing = {}, {}, {}
    plant = ctrl.solver
    train_runs[0] = run_evaluation(ctrl.prior_ctrl, x0, episode_len, tstep0, plant_solver=plant)
    test_runs[0] = run_evaluation(ctrl.prior_ctrl, x0, episode_len, tstep0, plant_solver=plant)
    x_train = np.zeros((0, sum(spec.gp_dims)))
    y_train = np.zeros((0, spec.n_gp))
    for epoch in range(1, n_epochs + 1):
        state, actions, next_state = sample_data(train_runs[epoch - 1], samples_per_epoch, rng)
        inputs, targets = ctrl.preprocess_data(state, actions, next_state)
        # every rank's new transitions, in rank order (one all-gather per epoch)
        inputs, targets = D.gather_rows(inputs), D.gather_rows(targets)
        x_train = np.vstack((x_train, inputs))
        y_train = np.vstack((y_train, targets))
        t3 = time.perf_counter()
        ctrl.train_gp(x=x_train, y=y_train, lr=lr, iterations=gp_iterations)
        t4 = time.perf_counter()
        test_runs[epoch] = run_evaluation(ctrl, x0, episode_len, tstep0)
        t5 = time.perf_counter()
        train_runs[epoch] = run_evaluation(ctrl, x0, episode_len, tstep0)
        t6 = time.perf_counter()
        timing[epoch] = {"train_gp": t4 - t3, "test": t5 - t4, "collect": t6 - t5, "n_train": len(x_train)}
    return train_runs, test_runs, timing


def get_runtime(test_runs: dict, train_runs: dict) -> dict:
    """Mean / std / max per-step inference time per epoch, first step dropped
    (`gpmpc/plotting.py:10-37`)."""
    epochs = sorted(test_runs)
    mean = np.zeros(len(epochs))
    std = np.zeros(len(epochs))
    mx = np.zeros(len(epochs))
    n_train = []
    for i, e in enumerate(epochs):
        rt = np.asarray(test_runs[e]["inference_time_data"][1:])
        mean[i], std[i], mx[i] = rt.mean(), rt.std(), rt.max()
        n_train.append(int(np.prod(train_runs[e]["action"].shape[:2])))
    return {"mean": mean, "std": std, "max": mx, "num_train_samples": n_train}


def save_runtime_csv(runtime: dict, num_points_per_epoch, save_dir: Path) -> Path:
    """runtime.csv with the reference's columns (`gpmpc/plotting.py:61-62`)."""
    save_dir = Path(save_dir)
    save_dir.mkdir(parents=True, exist_ok=True)
    data = np.vstack((num_points_per_epoch, runtime["mean"], runtime["std"], runtime["max"])).T
    path = save_dir / "runtime.csv"
    np.savetxt(path, data, delimiter=",", header="Train Steps, Mean, Std, Max")
    return path
