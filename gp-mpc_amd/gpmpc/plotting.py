"""Result figures and CSVs of the learning loop (`gpmpc/plotting.py`).

Host-side reporting only (matplotlib, Agg backend; nothing here touches the GPU).  The runs are
the dicts :func:`gpmpc.learning.run_evaluation` returns, batched over instances: ``obs``
(steps+1, B, nx), ``action`` (steps, B, nu), ``inference_time_data`` (steps,).  The reference
plots its single episode; here ``instance`` selects which of the B episodes is drawn (a 2-D
``obs`` (steps+1, nx), the reference's layout, is accepted as well).

* :func:`plot_runtime`        -- mean +- std and max inference time per epoch (`plotting.py:40-62`)
* :func:`plot_runs`           -- one state over the epochs vs the reference (`plotting.py:65-86`)
* :func:`plot_runs_input`     -- one input over the epochs (`plotting.py:89-104`)
* :func:`plot_learning_curve` -- figure + CSV of a per-epoch scalar (`plotting.py:107-120`)
* :func:`plot_path`           -- position paths in the model's planes (`plotting.py:121-155`,
  generalised from the 3D quadrotor's x-y / x-z / y-z planes to quad2d's x-z and cartpole's x-theta)
* :func:`make_plots`          -- the per-run figure set (`plotting.py:158-181`, ``make_quad_plots``)
* :func:`plot_state_eval`     -- states vs reference over time (`plotting.py:184-228`)
"""

from __future__ import annotations

from pathlib import Path

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402
from matplotlib.ticker import FormatStrFormatter  # noqa: E402

from .learning import get_runtime, save_runtime_csv  # noqa: E402

STATE_LABELS = {
    "quad3d": ["x", "d_x", "y", "d_y", "z", "d_z", "phi", "theta", "psi", "d_phi", "d_theta", "d_psi"],
    "quad2d": ["x", "d_x", "z", "d_z", "theta", "d_theta"],
    "cartpole": ["x", "d_x", "theta", "d_theta"],
}
# position planes per model: (title, x index, y index, x label, y label)
PATH_PLANES = {
    "quad3d": [("X-Y plane path", 0, 2, "X [m]", "Y [m]"), ("X-Z plane path", 0, 4, "X [m]", "Z [m]"),
               ("Y-Z plane path", 2, 4, "Y [m]", "Z [m]")],
    "quad2d": [("X-Z plane path", 0, 2, "X [m]", "Z [m]")],
    "cartpole": [("cart position vs pole angle", 0, 2, "x [m]", "theta [rad]")],
}


def _episode(run: dict, key: str, instance: int) -> np.ndarray:
    a = np.asarray(run[key])
    return a[:, instance, :] if a.ndim == 3 else a


def _label(epoch: int) -> str:
    return "prior MPC" if epoch == 0 else f"GP-MPC {epoch}"


def _finish(fig, path: Path | None):
    if path is not None:
        fig.savefig(path)
    plt.close(fig)


def plot_runtime(runtime: dict, num_points_per_epoch, save_dir: Path) -> Path:
    """Inference time per epoch (mean +- std band, max) and ``runtime.csv``."""
    save_dir = Path(save_dir)
    save_dir.mkdir(parents=True, exist_ok=True)
    n = np.asarray(num_points_per_epoch)
    mean, std = np.asarray(runtime["mean"]), np.asarray(runtime["std"])
    fig, ax = plt.subplots()
    ax.plot(n, mean, label="mean")
    ax.fill_between(n, mean - std, mean + std, alpha=0.3, label="1-std")
    ax.plot(n, runtime["max"], label="max", color="r")
    ax.set_xlabel("Train Steps")
    ax.set_ylabel("Runtime (s) ")
    ax.legend()
    _finish(fig, save_dir / "runtime.png")
    return save_runtime_csv(runtime, n, save_dir)


def _plot_series(runs, num_epochs, key, ind, ylabel, save_path, instance, traj=None):
    fig, ax = plt.subplots()
    if traj is not None:
        ax.plot(np.asarray(traj)[:, ind], label="Reference", color="gray", linestyle="--")
    for epoch in range(num_epochs):
        ax.plot(_episode(runs[epoch], key, instance)[:, ind], label=_label(epoch))
    ax.set_title(ylabel)
    ax.set_xlabel("Step")
    ax.set_ylabel(ylabel)
    ax.legend()
    _finish(fig, save_path)


def plot_runs(all_runs: dict, num_epochs: int, ind: int = 0, ylabel: str = "x position",
              save_dir: Path | None = None, traj: np.ndarray | None = None, instance: int = 0):
    """State ``ind`` of each epoch's episode, with the reference (traj (steps, nx)) if given."""
    path = Path(save_dir) / f"x{ind}.png" if save_dir is not None else None
    _plot_series(all_runs, num_epochs, "obs", ind, ylabel, path, instance, traj)


def plot_runs_input(all_runs: dict, num_epochs: int, ind: int = 0, ylabel: str = "x position",
                    save_dir: Path | None = None, instance: int = 0):
    """Input ``ind`` of each epoch's episode."""
    path = Path(save_dir) / f"u{ind}.png" if save_dir is not None else None
    _plot_series(all_runs, num_epochs, "action", ind, ylabel, path, instance)


def plot_learning_curve(avg_rewards, num_points_per_epoch, stem: str, save_dir: Path) -> Path:
    """A per-epoch scalar over the number of training samples: ``<stem>.png`` and ``<stem>.csv``."""
    save_dir = Path(save_dir)
    save_dir.mkdir(parents=True, exist_ok=True)
    fig, ax = plt.subplots()
    ax.plot(num_points_per_epoch, avg_rewards)
    ax.set_title("Avg Episode" + stem)
    ax.set_xlabel("Training Steps")
    ax.set_ylabel(stem)
    _finish(fig, save_dir / (stem + ".png"))
    path = save_dir / (stem + ".csv")
    np.savetxt(path, np.vstack((num_points_per_epoch, avg_rewards)).T, delimiter=",", header="Train steps,Cost")
    return path


def plot_path(runs: dict, ref: np.ndarray, model: str, save_dir: Path, instance: int = 0) -> Path:
    """Position paths of every epoch in the model's planes (``xyz_path.png``); ref (steps, nx)."""
    planes = PATH_PLANES[model]
    fig, axes = plt.subplots(len(planes), 1, squeeze=False)
    for ax, (title, i, j, xl, yl) in zip(axes[:, 0], planes):
        ax.plot(ref[:, i], ref[:, j], label="Reference", color="gray", linestyle="--")
        for epoch in range(len(runs)):
            obs = _episode(runs[epoch], "obs", instance)
            ax.plot(obs[:, i], obs[:, j], label=_label(epoch))
        ax.set_title(title)
        ax.set_xlabel(xl)
        ax.set_ylabel(yl)
        ax.legend()
    path = Path(save_dir) / "xyz_path.png"
    _finish(fig, path)
    return path


def make_plots(test_runs: dict, train_runs: dict, trajectory: np.ndarray, save_dir: Path, model: str,
               instance: int = 0) -> Path:
    """The reference's per-run figure set under ``save_dir/figs``: paths, every state and input
    over the epochs, and the runtime figure + CSV.  ``trajectory`` is (L, nx), trimmed to the
    episode length.  The sample count of epoch e is the transitions collected in the train
    episodes of epochs 1..e (all instances)."""
    obs0 = np.asarray(test_runs[0]["obs"])
    num_steps, nx = obs0.shape[0], obs0.shape[-1]
    nu = np.asarray(test_runs[0]["action"]).shape[-1]
    trajectory = np.asarray(trajectory)[:num_steps]
    num_epochs = len(test_runs)
    fig_dir = Path(save_dir) / "figs"
    fig_dir.mkdir(parents=True, exist_ok=False)
    plot_path(test_runs, trajectory, model, fig_dir, instance)
    for ind in range(nx):
        plot_runs(test_runs, num_epochs, ind=ind, ylabel=f"x{ind}", save_dir=fig_dir, traj=trajectory, instance=instance)
    for ind in range(nu):
        plot_runs_input(test_runs, num_epochs, ind=ind, ylabel=f"u{ind}", save_dir=fig_dir, instance=instance)
    points, per_epoch = 0, [0]
    for epoch in range(1, num_epochs):
        points += int(np.prod(np.asarray(train_runs[epoch]["action"]).shape[:-1]))
        per_epoch.append(points)
    plot_runtime(get_runtime(test_runs, train_runs), per_epoch, fig_dir)
    return fig_dir


def plot_state_eval(trajectories: dict, reference: np.ndarray, dt: float, save_path: Path, model: str,
                    instance: int = 0) -> Path:
    """States of one episode against the reference (nx, L) over time: ``state_trajectories.png``."""
    states = _episode(trajectories, "obs", instance)
    inputs = _episode(trajectories, "action", instance)
    nx = states.shape[1]
    labels = STATE_LABELS[model]
    if len(labels) != nx:
        raise ValueError(f"{model} has {len(labels)} states, the run has {nx}")
    n = min(inputs.shape[0], states.shape[0])
    times = np.linspace(0, dt * n, n)
    fig, axs = plt.subplots(nx, figsize=(8, nx * 1), squeeze=False)
    axs = axs[:, 0]
    for k in range(nx):
        axs[k].plot(times, states[:n, k], label="actual")
        axs[k].plot(times, reference[k, :n], color="r", label="desired")
        axs[k].set(ylabel=labels[k])
        axs[k].yaxis.set_major_formatter(FormatStrFormatter("%.1f"))
        if k != nx - 1:
            axs[k].set_xticks([])
    axs[0].set_title("State Trajectories")
    axs[-1].legend(ncol=3, bbox_transform=fig.transFigure, bbox_to_anchor=(1, 0), loc="lower right")
    axs[-1].set(xlabel="time (sec)")
    fig.tight_layout()
    path = Path(save_path) / "state_trajectories.png"
    _finish(fig, path)
    return path
