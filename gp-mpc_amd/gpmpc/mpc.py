"""Nominal MPC with the prior model only (drop-in for ``gpmpc/mpc.py``).

Same batched HIP solver as :class:`gpmpc.gpmpc.GPMPC` with the GP residual and the
tightening disabled and the reference's ``uh = +1e-8`` constraint offset
(`gpmpc/mpc.py:157-162`).  ``q_mpc`` / ``r_mpc`` are the diagonals of the LINEAR_LS weights
W = blkdiag(Q, R), W_e = Q (`gpmpc/mpc.py:42-45,101-102`).  ``reset()`` also resets the solver
iterate, as the reference calls ``acados_solver.reset()`` (`gpmpc/mpc.py:60-63`).
"""

from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from .models import ModelSpec, get_spec
from .solver import BatchSolver, STATUS_NAMES


class MPC:
    """MPC with the full nonlinear prior model (`gpmpc/mpc.py:12-193`)."""

    # the reference's quadrotor hover input (`gpmpc/mpc.py:15`); an instance's U_EQ is its model's
    U_EQ: np.ndarray = np.array([0.3234, 0, 0, 0])

    def __init__(self, symbolic_model, traj: np.ndarray | None = None, q_mpc: list | None = None,
                 r_mpc: list | None = None, output_dir: Path | None = None, horizon: int = 5, device: str = "cuda",
                 batch: int = 1, **solver_kw):
        spec = (symbolic_model if isinstance(symbolic_model, ModelSpec) else get_spec(symbolic_model)).copy()
        if q_mpc is not None:   # `gpmpc/mpc.py:42-45`: Q = diag(q_mpc), R = diag(r_mpc)
            assert len(q_mpc) == spec.nx
            spec.q_diag = np.asarray(q_mpc, dtype=np.float64).copy()
        if r_mpc is not None:
            assert len(r_mpc) == spec.nu
            spec.r_diag = np.asarray(r_mpc, dtype=np.float64).copy()
        self.model = spec
        self.U_EQ = spec.u_eq.copy()
        self.Q, self.R = np.diag(spec.q_diag), np.diag(spec.r_diag)
        self.T = int(horizon)
        self.traj = spec.reference_trajectory() if traj is None else np.asarray(traj, dtype=np.float64)
        self.traj_step = 0
        self.u_ref = np.repeat(self.U_EQ[..., None], self.T, axis=-1)
        self.output_dir = output_dir
        self.device = torch.device(device)
        self.batch = int(batch)
        self._solver = None
        self._solver_kw = solver_kw
        self._tstep = None

    @property
    def solver(self) -> BatchSolver:
        # built lazily: GPMPC constructs its prior controller eagerly like the reference,
        # but the GPU handle is only created when the prior controller is used.
        if self._solver is None:
            self._solver = BatchSolver(self.model, self.T, self.batch, device=self.device, traj=self.traj, uh=1e-8,
                                       **self._solver_kw)
            self._solver.set_gps(None)
            self._solver.set_tightening(False)
            self._tstep = torch.zeros(self.batch, dtype=torch.int32, device=self.device)
        return self._solver

    def reset(self):
        """Prepares for training or evaluation (`gpmpc/mpc.py:60-63`)."""
        self.solver.reset(reset_iterate=True)
        self.traj_step = 0

    def select_action(self, obs: np.ndarray) -> np.ndarray:
        """`gpmpc/mpc.py:172-186`."""
        assert self.batch == 1, "select_action is the single-instance form; use select_action_batch"
        s = self.solver
        x0 = torch.as_tensor(np.asarray(obs, dtype=np.float64).reshape(1, -1), device=self.device)
        self._tstep.fill_(self.traj_step)
        self.traj_step += 1
        u0 = s.solve(x0, self._tstep)
        status = int(s.status[0].item())
        assert status in [0, 2], f"solver returned unexpected status {status} ({STATUS_NAMES.get(status)})."
        return u0[0].cpu().numpy()

    def select_action_batch(self, obs: torch.Tensor, tstep: torch.Tensor | None = None) -> torch.Tensor:
        s = self.solver
        if tstep is None:
            self._tstep.fill_(self.traj_step)
            tstep = self._tstep
            self.traj_step += 1
        return s.solve(obs, tstep)

    def reference_trajectory(self) -> np.ndarray:
        """`gpmpc/mpc.py:188-193`."""
        indices = np.arange(self.traj_step, self.traj_step + self.T + 1) % self.traj.shape[-1]
        return self.traj[:, indices]

    @staticmethod
    def setup_constraints(sym, low, high):
        """`gpmpc/mpc.py:165-170`."""
        dim = low.shape[0]
        A = np.vstack((-np.eye(dim), np.eye(dim)))
        b = np.hstack((-low, high))
        return A @ sym - b
