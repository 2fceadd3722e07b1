"""Batched solver handle: B independent GP-MPC instances on one MI355X.

Thin host layer over the C ABI (``include/gpmpc_mi355x.h``): it owns the solver handle,
uploads the OCP definition and the GP replicas, and runs one batched control step per
:meth:`BatchSolver.solve` (one ``gpmpc_solve`` call = the variance kernel + the SQP kernel,
asynchronous on torch's current stream).  All per-step tensors stay on the device.
"""

from __future__ import annotations

import ctypes

import numpy as np
import scipy.linalg
import scipy.stats
import torch

from . import _lib
from .gp import LOVE_CHOLESKY_ROWS, GaussianProcess
from .models import ModelSpec

STATUS_NAMES = {0: "SUCCESS", 1: "NAN_DETECTED", 2: "MAXITER", 3: "MINSTEP", 4: "QP_FAILURE"}


def discretize_linear_system(A, B, dt: float, exact: bool = False):
    """(Exact) ZOH discretisation (`gpmpc/gpmpc.py:517-527`)."""
    nx, nu = A.shape[1], B.shape[1]
    if exact:
        M = np.zeros((nx + nu, nx + nu))
        M[:nx, :nx] = A
        M[:nx, nx:] = B
        Md = scipy.linalg.expm(M * dt)
        return Md[:nx, :nx], Md[:nx, nx:]
    return np.eye(nx) + A * dt, B * dt


def setup_prior_dynamics(dfdx, dfdu, Q, R, dt):
    """LQR gain of the discretised prior (`gpmpc/gpmpc.py:500-507`)."""
    A, B = discretize_linear_system(dfdx, dfdu, dt, exact=True)
    P = scipy.linalg.solve_discrete_are(A, B, Q, R)
    btp = B.T @ P
    lqr_gain = -np.linalg.inv(R + btp @ B) @ (btp @ A)
    return A, B, lqr_gain


def inverse_cdf(prob: float, nx: int) -> float:
    """`gpmpc/gpmpc.py:63-65`."""
    return float(scipy.stats.norm.ppf(1 - (1 / nx - (prob + 1) / (2 * nx))))


def _c(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


class BatchSolver:
    """One solver handle for ``batch`` instances of ``spec`` with horizon ``horizon``."""

    def __init__(self, spec: ModelSpec, horizon: int, batch: int, device="cuda", prior_params: dict | None = None,
                 traj: np.ndarray | None = None, uh: float = -1e-8, cost_scaling: bool = True, max_iter: int = 25,
                 tol: float = 1e-6, qp_max_iter: int = 50, qp_tol: float | None = None, qp_mu0: float = 1.0):
        self.lib = _lib.load()
        self.spec = spec
        self.H = int(horizon)
        self.batch = int(batch)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise _lib.GPMPCError("BatchSolver runs on the GPU (device must be cuda)")
        self.dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", self.dev_index)
        self.nx, self.nu = spec.nx, spec.nu
        h = ctypes.c_void_p()
        _lib.check(self.lib.gpmpc_create(spec.model_id, self.H, self.batch, self.dev_index, ctypes.byref(h)))
        self._h = h
        self._uh, self._cost_scaling = float(uh), int(cost_scaling)
        self.set_prior(prior_params)
        self.set_options(max_iter=max_iter, tol=tol, qp_max_iter=qp_max_iter, qp_tol=qp_tol, qp_mu0=qp_mu0)
        self.set_reference(spec.reference_trajectory() if traj is None else traj)
        self.set_var_inputs(spec.var_inputs)
        self.gps: list[GaussianProcess] | None = None
        # per-step device buffers
        kw = dict(device=self.device)
        B = self.batch
        self.u0 = torch.zeros(B, self.nu, dtype=torch.float64, **kw)
        self.status = torch.zeros(B, dtype=torch.int32, **kw)
        self.sqp_iter = torch.zeros(B, dtype=torch.int32, **kw)
        self.qp_iter = torch.zeros(B, dtype=torch.int32, **kw)
        self.res = torch.zeros(B, 4, dtype=torch.float64, **kw)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None:
            _lib._lib.gpmpc_destroy(h)
            self._h = None

    # ------------------------------------------------------------------ configuration
    def set_prior(self, prior_params: dict | None = None):
        """Prior model parameters (``spec.prior`` updated by ``prior_params``), bounds, weights."""
        spec = self.spec
        self.prior = dict(spec.prior if prior_params is None else {**spec.prior, **prior_params})
        params = _c(spec.param_vector(self.prior))
        self._keep = [params]
        _lib.check(self.lib.gpmpc_set_model(
            self._h, params.ctypes.data, params.size, spec.dt, _c(spec.x_lo).ctypes.data, _c(spec.x_hi).ctypes.data,
            _c(spec.u_lo).ctypes.data, _c(spec.u_hi).ctypes.data, _c(spec.q_diag).ctypes.data,
            _c(spec.r_diag).ctypes.data, _c(spec.u_eq).ctypes.data, self._uh, self._cost_scaling))

    def set_options(self, max_iter=25, tol=1e-6, qp_max_iter=50, qp_tol=None, qp_mu0=1.0):
        """SQP / QP options (gpmpc_set_options).  ``qp_tol=None``: the QP solves to the NLP tolerance,
        as acados passes its NLP tolerances on to the QP solver when the OCP leaves the QP
        tolerances unset (`gpmpc/gpmpc.py:257-263`)."""
        qp_tol = tol if qp_tol is None else qp_tol
        _lib.check(self.lib.gpmpc_set_options(self._h, int(max_iter), tol, tol, tol, tol, int(qp_max_iter), qp_tol, qp_mu0))

    def set_reference(self, traj: np.ndarray):
        traj = _c(traj)
        if traj.ndim != 2 or traj.shape[0] != self.nx:
            raise ValueError(f"reference trajectory must be (nx={self.nx}, L)")
        self.traj = traj
        _lib.check(self.lib.gpmpc_set_reference(self._h, traj.ctypes.data, traj.shape[1]))

    def set_gps(self, gps: list[GaussianProcess] | None, with_variance: bool = True, fitc: list | None = None,
                variance: str = "exact", love_rank: int = 100, love_force: bool = False):
        """Upload GP replicas.  ``fitc[g] = (S (M,d), w (M,))`` replaces GP g's mean by the FITC
        approximation (the variance stays exact, as in `gpmpc/gpmpc.py:441-445`).

        ``variance="love"``: the tightening variance of GPs with more than
        ``LOVE_CHOLESKY_ROWS`` (800) training rows uses the rank-``love_rank`` Lanczos root
        (`GaussianProcess.love_root`), as gpytorch's ``fast_pred_var`` does in the reference
        (`gpmpc/gpmpc.py:442-444`); smaller GPs keep the exact root, like gpytorch's Cholesky
        path.  ``love_force`` applies the Lanczos root at every size (tests)."""
        if variance not in ("exact", "love"):
            raise ValueError("variance must be 'exact' or 'love'")
        self.love_ranks = [None] * self.spec.n_gp   # columns of each GP's LOVE root (None: exact)
        self.love_roots = [None] * self.spec.n_gp   # the uploaded roots (host, float64), for checkers
        if gps is None:
            _lib.check(self.lib.gpmpc_use_gp(self._h, 0))
            self.gps = None
            return
        if len(gps) != self.spec.n_gp:
            raise ValueError(f"{self.spec.name} needs {self.spec.n_gp} GPs")
        for g, gp in enumerate(gps):
            lay = gp.device_layout("cpu")
            X = _c(gp.train_inputs[0].cpu().numpy())
            Linv = _c(lay["Linv"].cpu().numpy()) if with_variance else None
            if fitc is not None and fitc[g] is not None:
                S, w = _c(fitc[g][0]), _c(fitc[g][1])
                _lib.check(self.lib.gpmpc_set_gp(self._h, g, S.shape[0], S.shape[1], S.ctypes.data, w.ctypes.data,
                                                 X.shape[0], X.ctypes.data, None if Linv is None else Linv.ctypes.data,
                                                 gp.lengthscale, gp.outputscale, gp.noise))
            else:
                alpha = _c(lay["alpha"].cpu().numpy())
                _lib.check(self.lib.gpmpc_set_gp(self._h, g, X.shape[0], X.shape[1], X.ctypes.data, alpha.ctypes.data,
                                                 0, None, None if Linv is None else Linv.ctypes.data,
                                                 gp.lengthscale, gp.outputscale, gp.noise))
            if with_variance and variance == "love" and (love_force or X.shape[0] > LOVE_CHOLESKY_ROWS):
                R = _c(gp.love_root(love_rank).cpu().numpy())
                _lib.check(self.lib.gpmpc_set_gp_variance_root(self._h, g, R.shape[0], R.shape[1], R.ctypes.data))
                self.love_ranks[g] = R.shape[1]
                self.love_roots[g] = R
        _lib.check(self.lib.gpmpc_use_gp(self._h, 1))
        self.gps = gps

    def gp_mean_grad(self, gp_id: int, z: torch.Tensor):
        """GP mean (P,) and input gradient (P, d) at z (P, d) through the linearisation's MFMA tile
        sums (the casadi mean + AD of `gpmpc/gp.py:72-85`, `gpmpc/gpmpc.py:189-209`)."""
        z = z.to(self.device, torch.float64).contiguous()
        P = z.shape[0]
        mean = torch.empty(P, dtype=torch.float64, device=self.device)
        grad = torch.empty(P, z.shape[1], dtype=torch.float64, device=self.device)
        _lib.check(self.lib.gpmpc_gp_mean_grad(self._h, int(gp_id), z.data_ptr(), P, mean.data_ptr(),
                                               grad.data_ptr(), self._stream()))
        return mean, grad

    def set_var_inputs(self, var_inputs):
        """Per-GP input map of the tightening variance (indices into z = [x; u]); see
        gpmpc_set_var_inputs.  ``spec.var_inputs`` (the reference's map) is the default."""
        for g, idx in enumerate(var_inputs):
            a = np.ascontiguousarray(idx, dtype=np.int32)
            _lib.check(self.lib.gpmpc_set_var_inputs(self._h, g, a.ctypes.data, len(a)))

    def set_tightening(self, enabled: bool, prob: float = 0.95, Ad=None, Bd=None, K=None):
        if not enabled:
            _lib.check(self.lib.gpmpc_set_tightening(self._h, 0, 0.0, None, None, None))
            return
        Ad, Bd, K = _c(Ad), _c(Bd), _c(K)
        self._keep += [Ad, Bd, K]
        _lib.check(self.lib.gpmpc_set_tightening(self._h, 1, inverse_cdf(prob, self.nx), Ad.ctypes.data,
                                                 Bd.ctypes.data, K.ctypes.data))

    STATS_SLOTS = 12

    def set_stats(self, buf: torch.Tensor | None):
        """Device int64 (B, 10) accumulator of SQP/QP iteration sums, status counts and the
        largest SQP / QP iteration counts of one solve (or None); see gpmpc_set_stats_buffer."""
        if buf is not None:
            assert buf.shape == (self.batch, self.STATS_SLOTS) and buf.dtype == torch.int64 and buf.device == self.device
        self._stats = buf
        _lib.check(self.lib.gpmpc_set_stats_buffer(self._h, None if buf is None else buf.data_ptr(), self.STATS_SLOTS))

    def set_launch(self, waves: int = 0):
        """SQP-kernel launch shape (gpmpc_set_launch): waves per instance (0 auto, 1, 2, 4; quad3d:
        0 or 4).  A performance option; results agree to rounding."""
        _lib.check(self.lib.gpmpc_set_launch(self._h, int(waves)))

    def launch_info(self) -> dict:
        """What a solve of this batch runs (gpmpc_get_launch_info, gpmpc_get_launch_segments): SQP
        waves per instance, horizon segments of its Newton solves, and whether a step with a variance
        launch runs as overlapped halves (then the profiling events bracket spans of the step, not
        single kernels)."""
        w, o, g = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self.lib.gpmpc_get_launch_info(self._h, self.batch, ctypes.byref(w), ctypes.byref(o)))
        _lib.check(self.lib.gpmpc_get_launch_segments(self._h, self.batch, ctypes.byref(g)))
        return {"waves": w.value, "segments": g.value, "overlapped": o.value == 1, "tail_boost": o.value == 2}

    def set_tuning(self, **opts):
        """Performance switches (gpmpc_set_tuning): lin_cache=0/1, order=0/1/2, overlap=0/1,
        var_split=0/1/4, event_fence=0/1, seg=0/1, tail=K, seg_pivot=k.  Outputs do not depend on them (A/B knobs)."""
        for k, v in opts.items():
            if k not in _lib.TUNE:
                raise ValueError(f"unknown tuning option {k!r} (one of {sorted(_lib.TUNE)})")
            _lib.check(self.lib.gpmpc_set_tuning(self._h, _lib.TUNE[k], int(v)))

    def set_cost_output(self, enabled: bool = True) -> torch.Tensor | None:
        """Per-stage LINEAR_LS costs of every solve's new solution into ``self.stage_cost`` (B, H+1)
        (gpmpc_set_cost_buffer): 1/2 ||y_k - y_ref,k||^2_W with dt-scaled stage weights and the
        unscaled terminal weight (`gpmpc/gpmpc.py:231-239`); NaN for a failed solve."""
        self.stage_cost = (torch.full((self.batch, self.H + 1), float("nan"), dtype=torch.float64, device=self.device)
                           if enabled else None)
        _lib.check(self.lib.gpmpc_set_cost_buffer(self._h, None if self.stage_cost is None
                                                  else self.stage_cost.data_ptr()))
        return self.stage_cost

    def set_profiling(self, enabled: bool):
        _lib.check(self.lib.gpmpc_set_profiling(self._h, int(enabled)))

    def kernel_times(self) -> dict:
        """Summed HIP-event milliseconds of the variance / SQP kernels since the last call."""
        vm, sm = ctypes.c_double(), ctypes.c_double()
        vn, sn = ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self.lib.gpmpc_kernel_times(self._h, ctypes.byref(vm), ctypes.byref(vn), ctypes.byref(sm),
                                               ctypes.byref(sn)))
        return {"var_ms": vm.value, "var_launches": vn.value, "sqp_ms": sm.value, "sqp_launches": sn.value}

    def kernel_time_list(self, cap: int = 4096) -> dict:
        """Per-launch HIP-event milliseconds of the variance / SQP kernels since the last call."""
        vm = (ctypes.c_double * cap)()
        sm = (ctypes.c_double * cap)()
        vn, sn = ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self.lib.gpmpc_kernel_time_list(self._h, cap, vm, ctypes.byref(vn), sm, ctypes.byref(sn)))
        return {"var_ms": list(vm[:min(vn.value, cap)]), "sqp_ms": list(sm[:min(sn.value, cap)])}

    # ------------------------------------------------------------------ stepping
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def reset(self, reset_iterate: bool = False):
        _lib.check(self.lib.gpmpc_reset(self._h, self.batch, int(reset_iterate), self._stream()))

    def set_iterate(self, x: torch.Tensor, u: torch.Tensor):
        x = x.to(self.device, torch.float64).contiguous()
        u = u.to(self.device, torch.float64).contiguous()
        assert x.shape == (self.batch, self.H + 1, self.nx) and u.shape == (self.batch, self.H, self.nu)
        _lib.check(self.lib.gpmpc_set_iterate(self._h, self.batch, x.data_ptr(), u.data_ptr(), self._stream()))
        torch.cuda.current_stream(self.device).synchronize()

    def solve(self, x0: torch.Tensor, tstep: torch.Tensor) -> torch.Tensor:
        """One batched select_action: returns u0 (B, nu); status etc. in the buffers."""
        if x0.shape != (self.batch, self.nx) or x0.dtype != torch.float64 or x0.device != self.device:
            raise ValueError(f"x0 must be a ({self.batch}, {self.nx}) float64 tensor on {self.device}")
        if tstep.shape != (self.batch,) or tstep.dtype != torch.int32 or tstep.device != self.device:
            raise ValueError(f"tstep must be a ({self.batch},) int32 tensor on {self.device}")
        x0 = x0.contiguous()
        _lib.check(self.lib.gpmpc_solve(self._h, self.batch, x0.data_ptr(), tstep.data_ptr(), self.u0.data_ptr(),
                                        self.status.data_ptr(), self.sqp_iter.data_ptr(), self.qp_iter.data_ptr(),
                                        self.res.data_ptr(), self._stream()))
        return self.u0

    def solution(self):
        x = torch.empty(self.batch, self.H + 1, self.nx, dtype=torch.float64, device=self.device)
        u = torch.empty(self.batch, self.H, self.nu, dtype=torch.float64, device=self.device)
        t = torch.empty(self.batch, self.H + 1, self.nx + self.nu, dtype=torch.float64, device=self.device)
        _lib.check(self.lib.gpmpc_get_solution(self._h, self.batch, x.data_ptr(), u.data_ptr(), t.data_ptr(),
                                               self._stream()))
        return x, u, t

    def variance(self) -> torch.Tensor:
        """GP variances (B, H, n_gp) the last tightening used (gpmpc_get_variance): the variance
        kernel's output at the previous solution, likelihood noise included."""
        v = torch.empty(self.batch, self.H, self.spec.n_gp, dtype=torch.float64, device=self.device)
        _lib.check(self.lib.gpmpc_get_variance(self._h, self.batch, v.data_ptr(), self._stream()))
        return v

    def plant_step(self, x: torch.Tensor, u: torch.Tensor, tstep: torch.Tensor | None = None,
                   params: dict | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
        """Synthetic plant: RK4 of the prior-form model with ``params`` (default: spec.true_params)."""
        p = _c(self.spec.param_vector(self.spec.true_params if params is None else params))
        out = torch.empty_like(x) if out is None else out
        _lib.check(self.lib.gpmpc_plant_step(self._h, x.shape[0], p.ctypes.data, x.data_ptr(), u.data_ptr(),
                                             out.data_ptr(), None if tstep is None else tstep.data_ptr(),
                                             self._stream()))
        return out
