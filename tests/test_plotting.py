"""Result figures and CSVs (gpmpc/plotting.py, reference `gpmpc/plotting.py`): host-only, CPU."""

import numpy as np
import pytest

from gpmpc import plotting
from gpmpc.models import get_spec


def fake_runs(spec, epochs=3, steps=12, B=2, seed=0):
    rng = np.random.default_rng(seed)
    traj = spec.reference_trajectory().T
    runs = {}
    for e in range(epochs):
        runs[e] = {"obs": traj[: steps + 1, None, :] + 0.01 * rng.standard_normal((steps + 1, B, spec.nx)),
                   "action": rng.standard_normal((steps, B, spec.nu)),
                   "inference_time_data": 1e-3 * (1 + rng.random(steps))}
    return runs, traj


@pytest.mark.parametrize("name", ["quad3d", "quad2d", "cartpole"])
def test_make_plots_writes_reference_figure_set(tmp_path, name):
    spec = get_spec(name)
    test_runs, traj = fake_runs(spec)
    train_runs, _ = fake_runs(spec, seed=1)
    fig_dir = plotting.make_plots(test_runs, train_runs, traj, tmp_path, name, instance=1)
    names = {p.name for p in fig_dir.iterdir()}
    expected = {"xyz_path.png", "runtime.png", "runtime.csv"}
    expected |= {f"x{i}.png" for i in range(spec.nx)} | {f"u{i}.png" for i in range(spec.nu)}
    assert expected <= names
    rt = np.loadtxt(fig_dir / "runtime.csv", delimiter=",")
    # sample counts: 0, then the train transitions of epochs 1..e (12 steps x 2 instances each)
    np.testing.assert_array_equal(rt[:, 0], [0, 24, 48])
    # mean inference time drops the first step (gpmpc/plotting.py:25)
    np.testing.assert_allclose(rt[0, 1], test_runs[0]["inference_time_data"][1:].mean())
    with pytest.raises(FileExistsError):   # the reference refuses to overwrite a figure directory
        plotting.make_plots(test_runs, train_runs, traj, tmp_path, name)


def test_state_eval_and_learning_curve(tmp_path):
    spec = get_spec("quad2d")
    runs, traj = fake_runs(spec, epochs=1)
    p = plotting.plot_state_eval(runs[0], traj.T, spec.dt, tmp_path, "quad2d")
    assert p.exists() and p.stat().st_size > 0
    with pytest.raises(ValueError):
        plotting.plot_state_eval(runs[0], traj.T, spec.dt, tmp_path, "quad3d")
    csv = plotting.plot_learning_curve([3.0, 2.0, 1.5], [0, 100, 200], "cost", tmp_path)
    np.testing.assert_allclose(np.loadtxt(csv, delimiter=","), [[0, 3.0], [100, 2.0], [200, 1.5]])
    # the reference's single-episode layout (steps+1, nx) is accepted too
    single = {k: (v[:, 0] if v.ndim == 3 else v) for k, v in runs[0].items()}
    assert plotting.plot_state_eval(single, traj.T, spec.dt, tmp_path, "quad2d").exists()
