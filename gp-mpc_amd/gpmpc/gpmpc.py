"""GP-MPC controller on the MI355X (drop-in for ``gpmpc/gpmpc.py``).

:class:`GPMPC` keeps the reference's surface -- ``GPMPC(model, traj, prior_params, horizon,
q_mpc, r_mpc, sparse_gp, prob, max_gp_samples, seed, device)``, ``train_gp``, ``reset``,
``select_action(obs) -> action``, ``x_prev`` / ``u_prev``, ``prior_ctrl``,
``gaussian_process`` (`gpmpc/gpmpc.py:20-111,153-164,334-368`) -- and adds the batched
form ``select_action_batch(obs[B, nx]) -> actions[B, nu]`` on device tensors.  The
acados OCP (`gpmpc/gpmpc.py:166-320`) is replaced by the batched HIP solver
(``csrc/sqp_kernel.hip``); there is no code generation and no CPU fallback.

``model`` is a :class:`gpmpc.models.ModelSpec` or its name (``"quad3d"``, ``"quad2d"``,
``"cartpole"``); it takes the role of crazyflow's ``symbolic_attitude`` model object.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from . import _lib
from .gp import GaussianProcess, fit_gp
from .models import ModelSpec, get_spec
from .mpc import MPC
from .solver import BatchSolver, STATUS_NAMES, inverse_cdf, setup_prior_dynamics


class GPMPC:
    """Implements a GP-MPC controller on the MI355X HIP solver."""

    # the reference's quadrotor hover input (`gpmpc/gpmpc.py:18`); an instance's U_EQ is its model's
    U_EQ: np.ndarray = np.array([0.3234, 0, 0, 0])

    def __init__(self, symbolic_model, traj: np.ndarray | None = None, prior_params: dict | None = None,
                 horizon: int = 25, q_mpc: list | None = None, r_mpc: list | None = None, sparse_gp: bool = False,
                 prob: float = 0.955, max_gp_samples: int = 30, seed: int = 1337, device: str = "cuda",
                 output_dir: Path | None = None, batch: int = 1, variance_inputs: str = "reference",
                 variance: str = "love", **solver_kw):
        spec = (symbolic_model if isinstance(symbolic_model, ModelSpec) else get_spec(symbolic_model)).copy()
        # "reference": the variance input map of `gpmpc/gpmpc.py:437-444` (for quad3d it indexes the
        # full state-input vector with the GP-input-space indices); "dynamics": each GP's own inputs
        if variance_inputs == "dynamics":
            spec.var_inputs = spec.gp_inputs
        elif variance_inputs != "reference":
            raise ValueError("variance_inputs must be 'reference' or 'dynamics'")
        self.model = spec
        # tightening variance.  Default "love": what the reference computes -- its
        # propagate_constraint_limits runs under gpytorch.settings.fast_pred_var() (gpmpc.py:442-444),
        # i.e. the exact Cholesky variance up to gpytorch's max_cholesky_size (800 training rows)
        # and the rank-100 Lanczos (LOVE) root above it; "exact": L^-1 k at every size.
        self.variance = variance
        if q_mpc is not None:
            spec.q_diag = np.asarray(q_mpc, dtype=np.float64)
        if r_mpc is not None:
            spec.r_diag = np.asarray(r_mpc, dtype=np.float64)
        assert len(spec.q_diag) == spec.nx and len(spec.r_diag) == spec.nu
        if prior_params is not None:
            missing = [k for k in spec.prior if k not in prior_params]
            if missing:
                raise ValueError(f"GPMPC requires prior_params with keys {sorted(spec.prior)}; missing {missing}")
            spec.prior = {k: float(prior_params[k]) for k in spec.prior}
        self.sparse = sparse_gp
        self.output_dir = output_dir
        self.device = torch.device(device)
        self.dt = spec.dt
        self.T = int(horizon)
        self.Q, self.R = np.diag(spec.q_diag), np.diag(spec.r_diag)
        self.U_EQ = spec.u_eq.copy()
        self.traj = spec.reference_trajectory() if traj is None else np.asarray(traj, dtype=np.float64)
        self.ref_action = np.repeat(self.U_EQ[:, None], self.T, axis=1)
        self.traj_step = 0
        self.np_random = np.random.default_rng(seed)
        self.gp_idx = self._gp_columns(spec)
        # thrust map of the quadrotors (`gpmpc/gpmpc.py:45`); cartpole has none
        self.acc_symbolic_fn = self.setup_symbolic_acceleration(spec.prior) if "a" in spec.prior else None
        self.gaussian_process: list[GaussianProcess] | None = None
        self._requires_recompile = False
        self.prob = prob
        self.inverse_cdf = inverse_cdf(prob, spec.nx)
        self.max_gp_samples = max_gp_samples
        self.Bd = spec.bd_matrix()
        self.batch = int(batch)

        self.prior_ctrl = MPC(spec, traj=self.traj, horizon=self.T, q_mpc=list(spec.q_diag),
                              r_mpc=list(spec.r_diag), device=device, batch=batch, **solver_kw)
        dfdx, dfdu = spec.prior_jacobian(np.zeros(spec.nx), spec.u_eq)
        self.discrete_dfdx, self.discrete_dfdu, self.lqr_gain = setup_prior_dynamics(dfdx, dfdu, self.Q, self.R, self.dt)

        self.solver = BatchSolver(spec, self.T, self.batch, device=self.device, traj=self.traj, uh=-1e-8, **solver_kw)
        self.solver.set_tightening(True, prob, self.discrete_dfdx, self.discrete_dfdu, self.lqr_gain)
        self._x_prev = None
        self._u_prev = None
        self._has_prev = False
        self._tstep = torch.zeros(self.batch, dtype=torch.int32, device=self.device)
        # select_action's host staging: pinned buffers, so the observation / reference index go in and
        # the action / status come back as asynchronous copies with one synchronisation per call
        self._pinned = None
        if self.batch == 1 and torch.device(self.device).type == "cuda":
            self._pinned = (torch.empty(1, spec.nx, dtype=torch.float64, pin_memory=True),
                            torch.empty(1, dtype=torch.int32, pin_memory=True),
                            torch.empty(spec.nu, dtype=torch.float64, pin_memory=True),
                            torch.empty(1, dtype=torch.int32, pin_memory=True))
            self._x0_dev = torch.empty(1, spec.nx, dtype=torch.float64, device=self.device)

    @staticmethod
    def _gp_columns(spec: ModelSpec) -> list[list[int]]:
        """Column groups of the concatenated GP training inputs (`gpmpc/gpmpc.py:59`)."""
        cols, c = [], 0
        for d in spec.gp_dims:
            cols.append(list(range(c, c + d)))
            c += d
        return cols

    # ------------------------------------------------------------------ training data
    def setup_symbolic_acceleration(self, params: dict):
        """Prior thrust map T_c -> a T_c + b (`gpmpc/gpmpc.py:322-325`), a numpy callable."""
        a, b = float(params["a"]), float(params["b"])
        return lambda thrust_cmd: a * np.asarray(thrust_cmd, dtype=np.float64) + b

    def prior_dynamics(self, x: np.ndarray, u: np.ndarray) -> np.ndarray:
        """Continuous prior f(x, u) for rows of x (n, nx), u (n, nu) (crazyflow ``fc_func``)."""
        return self.model.prior_f(x, u)

    def preprocess_data(self, x: np.ndarray, u: np.ndarray, x_next: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """GP training inputs (N, sum d_g) and targets (N, n_gp) from transitions
        (`gpmpc/gpmpc.py:113-151`): numerically differentiated next state minus the prior.

        quad3d follows the reference literally, including its constants (g = 9.81 and
        dt = 1/60, not the model's dt) and the thrust target as the norm of the acceleration
        minus the prior thrust map.  quad2d / cartpole apply the same recipe to their GP
        outputs (thrust-acceleration norm and pitch rate; cart and pole accelerations).
        """
        x, u, x_next = (np.atleast_2d(np.asarray(a, dtype=np.float64)) for a in (x, u, x_next))
        spec = self.model
        if spec.name == "quad3d":
            g, dt = 9.81, 1 / 60
            x_dot = (x_next - x) / dt
            acc = np.sqrt(x_dot[:, 1] ** 2 + x_dot[:, 3] ** 2 + (x_dot[:, 5] + g) ** 2)
            acc_target = acc - self.acc_symbolic_fn(u[:, 0])
            f = self.prior_dynamics(x, u)
            phi_target = x_dot[:, 6] - f[:, 6]
            theta_target = x_dot[:, 7] - f[:, 7]
            inputs = np.column_stack([u[:, 0], x[:, 6], x[:, 9], u[:, 1], x[:, 7], x[:, 10], u[:, 2]])
            return inputs, np.column_stack([acc_target, phi_target, theta_target])
        dt = spec.dt
        x_dot = (x_next - x) / dt
        f = self.prior_dynamics(x, u)
        z = np.hstack([x, u])
        inputs = np.hstack([z[:, list(idx)] for idx in spec.gp_inputs])
        if spec.name == "quad2d":
            acc = np.sqrt(x_dot[:, 1] ** 2 + (x_dot[:, 3] + spec.gravity) ** 2)
            targets = np.column_stack([acc - self.acc_symbolic_fn(u[:, 0]), x_dot[:, 5] - f[:, 5]])
        else:  # cartpole: residual cart / pole accelerations
            targets = np.column_stack([x_dot[:, 1] - f[:, 1], x_dot[:, 3] - f[:, 3]])
        return inputs, targets

    # ------------------------------------------------------------------ GP management
    def train_gp(self, x: np.ndarray, y: np.ndarray, lr: float, iterations: int):
        """Fit one GP per output column on its input columns (`gpmpc/gpmpc.py:153-164`), on the
        controller's device (the MI355X); one all-reduce of the MLL gradient per Adam step
        when running data-parallel (gpmpc/distributed.py)."""
        x_train = torch.tensor(np.asarray(x, dtype=np.float64), device=self.device)
        y_train = torch.tensor(np.asarray(y, dtype=np.float64), device=self.device)
        gps = []
        from . import distributed as D

        _, size = D.world()
        if size > 1:   # the row-split gradient of fit_gp_allreduce is only valid on identical replicas
            D.assert_replicated(x, y)
        for i, idx in enumerate(self.gp_idx):
            gp = GaussianProcess(x_train[:, idx], y_train[:, i])
            if size > 1:   # data-parallel fit: one all-reduce of the MLL gradient per Adam step
                D.fit_gp_allreduce(gp, n_train=iterations, lr=lr)
            else:
                fit_gp(gp, n_train=iterations, lr=lr, device=self.device)
            gps.append(gp)
        self.set_gaussian_processes(gps)

    def set_gaussian_processes(self, gps: list[GaussianProcess]):
        for gp in gps:
            if gp.K is None:
                gp.K, gp.K_inv = gp.compute_covariances()
        self.gaussian_process = gps
        self._requires_recompile = True

    def precompute_sparse_posterior_mean(self, n_samples: int):
        """FITC weights on random training rows (`gpmpc/gpmpc.py:377-400`), computed where the
        GP lives (the MI355X for a GP fitted by ``train_gp``)."""
        gps = self.gaussian_process
        n = gps[0].train_inputs[0].shape[0]
        rand_idx = self.np_random.choice(range(n), size=n_samples, replace=False)
        out = []
        for gp in gps:
            X = gp.train_inputs[0]
            y = gp.train_targets
            S = X[torch.as_tensor(rand_idx, device=X.device)]
            with torch.no_grad():
                K = gp.K.to(X.device)
                K_ss = gp.kernel(S)
                K_xs = gp.kernel(X, S)
                Gamma = torch.diagonal(K) - (K_xs * torch.linalg.solve(K_ss, K_xs.T).T).sum(1)
                KG = K_xs.T / Gamma            # K_sx Lambda^-1 without the dense diagonal matrix
                Sigma_inv = K_ss + KG @ K_xs
                w = torch.linalg.solve(Sigma_inv, KG @ y)
            # the solver evaluates sf2 * sum_j w_j exp(.): the reference's covSE already carries sf2
            out.append((S.cpu().numpy(), w.cpu().numpy()))
        return out

    # ------------------------------------------------------------------ control
    def reset(self):
        """Reset before running (`gpmpc/gpmpc.py:94-111`): upload new GPs, forget x_prev/u_prev."""
        self.traj_step = 0
        self._tstep.zero_()
        if self._requires_recompile:
            assert self.gaussian_process is not None, "GP must be trained before reinitializing"
            fitc = None
            if self.sparse:
                n = self.gaussian_process[0].train_targets.shape[0]
                fitc = self.precompute_sparse_posterior_mean(min(n, self.max_gp_samples))
            self.solver.set_gps(self.gaussian_process, with_variance=True, fitc=fitc, variance=self.variance)
            self._requires_recompile = False
            # new GPs: the reference builds a fresh AcadosOcpSolver (`gpmpc/gpmpc.py:97-108`), whose
            # memory -- iterate and multipliers -- starts from zero
            self.solver.reset(reset_iterate=True)
        else:
            # same GPs: acados keeps its memory across episodes (`gpmpc/gpmpc.py:94-111` does not
            # reset the solver), so the first solve is warm-started from the last iterate
            self.solver.reset(reset_iterate=False)
        self._x_prev = None
        self._u_prev = None
        self._has_prev = False

    @property
    def x_prev(self):
        if not self._has_prev:
            return None
        if self._x_prev is None:
            x, u, _ = self.solver.solution()
            self._x_prev = x[0].T.cpu().numpy() if self.batch == 1 else x.cpu().numpy()
            self._u_prev = u[0].T.cpu().numpy() if self.batch == 1 else u.cpu().numpy()
        return self._x_prev

    @property
    def u_prev(self):
        if not self._has_prev:
            return None
        _ = self.x_prev
        return self._u_prev

    def select_action(self, obs: np.ndarray) -> np.ndarray:
        """Solve the nonlinear MPC problem to get the next action (`gpmpc/gpmpc.py:334-368`)."""
        assert not self._requires_recompile, "GP model must be uploaded (call reset())"
        assert self.gaussian_process is not None, "Gaussian processes are not initialized"
        assert self.batch == 1, "select_action is the single-instance form; use select_action_batch"
        if self._pinned is None:
            x0 = torch.as_tensor(np.asarray(obs, dtype=np.float64).reshape(1, -1), device=self.device)
            self._tstep.fill_(self.traj_step)
            self.traj_step += 1
            u0 = self.solver.solve(x0, self._tstep)
            status = int(self.solver.status[0].item())
            u = u0[0].cpu().numpy()
        else:
            x_h, t_h, u_h, s_h = self._pinned
            x_h.numpy()[0] = np.asarray(obs, dtype=np.float64).reshape(-1)
            t_h[0] = self.traj_step
            self.traj_step += 1
            self._x0_dev.copy_(x_h, non_blocking=True)
            self._tstep.copy_(t_h, non_blocking=True)
            u0 = self.solver.solve(self._x0_dev, self._tstep)
            u_h.copy_(u0[0], non_blocking=True)
            s_h.copy_(self.solver.status[:1], non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
            status = int(s_h[0])
            u = u_h.numpy().copy()
        assert status in [0, 2], f"solver returned unexpected status {status} ({STATUS_NAMES.get(status)})."
        self._has_prev = True
        self._x_prev = self._u_prev = None
        return u

    def select_action_batch(self, obs: torch.Tensor, tstep: torch.Tensor | None = None, check: bool = False):
        """Batched select_action on device tensors: obs (B, nx) float64 -> actions (B, nu).

        ``tstep`` (B,) int32 gives each instance's reference index (default: the shared
        ``traj_step`` counter).  ``check=True`` synchronises and asserts status in {0, 2}.
        """
        assert not self._requires_recompile, "GP model must be uploaded (call reset())"
        if tstep is None:
            self._tstep.fill_(self.traj_step)
            tstep = self._tstep
            self.traj_step += 1
        u0 = self.solver.solve(obs, tstep)
        self._has_prev = True
        self._x_prev = self._u_prev = None
        if check:
            bad = ~((self.solver.status == 0) | (self.solver.status == 2))
            if bool(bad.any()):
                i = int(torch.nonzero(bad)[0])
                raise AssertionError(f"instance {i}: unexpected status {int(self.solver.status[i])}")
        return u0

    def reference_trajectory(self) -> np.ndarray:
        """`gpmpc/gpmpc.py:509-514`."""
        indices = np.arange(self.traj_step, self.traj_step + self.T + 1) % self.traj.shape[-1]
        return self.traj[:, indices]

    @staticmethod
    def setup_constraints(sym, low, high):
        """Rows A sym - b of the box constraints (`gpmpc/gpmpc.py:327-332`)."""
        dim = low.shape[0]
        A = np.vstack((-np.eye(dim), np.eye(dim)))
        b = np.hstack((-low, high))
        return A @ sym - b

    setup_prior_dynamics = staticmethod(setup_prior_dynamics)
