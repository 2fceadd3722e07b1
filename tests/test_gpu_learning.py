"""End-to-end learning loop on the MI355X (`scripts/run_gp_mpc.py:86-137`): prior MPC episodes,
preprocess_data, GP fit on the GPU, GP-MPC episodes; batched synthetic plant."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.parametrize("sparse", [False, True])
def test_learn_loop_improves_tracking(sparse, tmp_path):
    torch = _torch()
    from gpmpc.gpmpc import GPMPC
    from gpmpc.learning import get_runtime, learn, save_runtime_csv, tracking_cost

    ctrl = GPMPC("quad2d", horizon=20, batch=32, sparse_gp=sparse, max_gp_samples=60, seed=3)
    train, test, timing = learn(n_epochs=2, ctrl=ctrl, lr=0.05, gp_iterations=60, seed=5, samples_per_epoch=150,
                                episode_len=40)
    for runs in (train, test):
        for e, d in runs.items():
            assert np.isin(d["status"], [0, 2]).all(), (e, np.unique(d["status"]))
    assert all(gp.train_inputs[0].device.type == "cuda" for gp in ctrl.gaussian_process)
    assert timing[2]["n_train"] == 300
    c0 = tracking_cost(test[0], ctrl.traj)
    c2 = tracking_cost(test[2], ctrl.traj)
    print(f"tracking cost prior {c0:.4e} -> GP-MPC epoch 2 {c2:.4e}")
    assert c2 < c0, (c0, c2)
    rt = get_runtime(test, train)
    path = save_runtime_csv(rt, [0, 150, 300], tmp_path)
    assert np.loadtxt(path, delimiter=",").shape == (3, 4)
