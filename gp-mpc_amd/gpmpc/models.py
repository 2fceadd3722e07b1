"""Model specifications for the GP-MPC solve path.

A model spec carries every constant the reference hard-codes for its one quadrotor
(SURVEY.md §2 "Hard-coded quadrotor specifics"), generalised so that the same solver
serves the three BASELINE.json model families:

* ``quad3d``  -- the reference's 12-state / 4-input attitude-interface quadrotor
  (`gpmpc/gpmpc.py:18,59,68,173,193-197,242-246`, `gpmpc/mpc.py:15,50-54`,
  `scripts/gp_mpc_config.yaml:7-17`).  The prior model comes from crazyflow's
  ``symbolic_attitude`` which is not installed; its equations are restated here
  (thrust map ``a*T_c+b``, roll ``c,d,e``, pitch ``f,h,l``; yaw assumed to reuse the
  roll coefficients so that (A,B) is stabilisable -- SURVEY.md §7 hard part (ii)).
* ``quad2d``  -- the build's planar (x-z) restriction of the same attitude model:
  state ``[x, vx, z, vz, theta, dtheta]``, input ``[T_c, P_c]``; GPs mirror the
  reference's thrust GP (input ``T_c``) and pitch GP (inputs ``theta, dtheta, P_c``).
* ``cartpole`` -- the build's cart-pole (gym equations, half pole length ``l``) with two
  residual GPs on the cart and pole accelerations, inputs ``[theta, dtheta, F]``.

Everything here is host-side configuration (numbers and index maps).  The dynamics
themselves are evaluated on the GPU by ``csrc/models.h``; the only host-side dynamics
code is the continuous-time prior Jacobian at the equilibrium, needed once at
construction for the LQR gain (`gpmpc/gpmpc.py:81-86,500-507`).
"""

from __future__ import annotations

import copy
from dataclasses import dataclass, field

import numpy as np

# Model ids shared with the C ABI (include/gpmpc_mi355x.h).
MODEL_QUAD2D = 0
MODEL_QUAD3D = 1
MODEL_CARTPOLE = 2

GRAVITY = 9.81

# Reference prior parameters, `scripts/gp_mpc_config.yaml:9-17`.
REF_PRIOR = dict(a=12.1432, b=1.8118, c=-72.08, d=-7.5755, e=39.8653, f=-72.08, h=-7.5755, l=39.8653)
# "True" plant parameters for synthetic data: the thrust map of the crazyflie attitude
# model hovers at U_EQ=0.3234 (a*0.3234+b = g); attitude coefficients are the prior's +20 %.
TRUE_QUAD = dict(a=20.907574256269616, b=3.653687545690674, c=-72.08 * 1.2, d=-7.5755 * 1.2,
                 e=39.8653 * 1.2, f=-72.08 * 1.2, h=-7.5755 * 1.2, l=39.8653 * 1.2)


@dataclass
class ModelSpec:
    name: str
    model_id: int
    nx: int
    nu: int
    dt: float
    prior: dict
    true_params: dict
    u_eq: np.ndarray
    x_lo: np.ndarray
    x_hi: np.ndarray
    u_lo: np.ndarray
    u_hi: np.ndarray
    q_diag: np.ndarray
    r_diag: np.ndarray
    gp_inputs: tuple          # per GP: indices into z = [x; u] used by the dynamics
    var_inputs: tuple         # per GP: indices into z used for the tightening variance
    unc_dims: tuple           # columns of I_nx forming Bd (`gpmpc/gpmpc.py:68-69`)
    gp_names: tuple = ()
    gravity: float = GRAVITY
    traj_len: int = 500
    extra: dict = field(default_factory=dict)

    # ------------------------------------------------------------------ parameters
    def param_vector(self, params: dict | None = None) -> np.ndarray:
        """Prior parameters in the order ``csrc/models.h`` reads them."""
        p = self.prior if params is None else params
        if self.model_id == MODEL_QUAD2D:
            v = [p["a"], p["b"], p["f"], p["h"], p["l"], self.gravity]
        elif self.model_id == MODEL_QUAD3D:
            v = [p["a"], p["b"], p["c"], p["d"], p["e"], p["f"], p["h"], p["l"], self.gravity]
        elif self.model_id == MODEL_CARTPOLE:
            v = [p["m_c"], p["m_p"], p["l"], self.gravity]
        else:
            raise ValueError(self.model_id)
        return np.asarray(v, dtype=np.float64)

    @property
    def n_gp(self) -> int:
        return len(self.gp_inputs)

    @property
    def gp_dims(self) -> tuple:
        return tuple(len(i) for i in self.gp_inputs)

    @property
    def n_unc(self) -> int:
        return len(self.unc_dims)

    def bd_matrix(self) -> np.ndarray:
        return np.eye(self.nx)[:, list(self.unc_dims)]

    # ------------------------------------------------------------------ prior Jacobian
    def prior_jacobian(self, x: np.ndarray, u: np.ndarray, params: dict | None = None):
        """Continuous-time prior Jacobians (dfdx, dfdu) -- the role of crazyflow's
        ``df_func`` at `gpmpc/gpmpc.py:81-83`."""
        p = self.prior if params is None else params
        nx, nu, g = self.nx, self.nu, self.gravity
        A = np.zeros((nx, nx))
        B = np.zeros((nx, nu))
        if self.model_id == MODEL_QUAD2D:
            th = x[4]
            acc = p["a"] * u[0] + p["b"]
            A[0, 1] = 1.0
            A[1, 4] = acc * np.cos(th)
            B[1, 0] = p["a"] * np.sin(th)
            A[2, 3] = 1.0
            A[3, 4] = -acc * np.sin(th)
            B[3, 0] = p["a"] * np.cos(th)
            A[4, 5] = 1.0
            A[5, 4] = p["f"]
            A[5, 5] = p["h"]
            B[5, 1] = p["l"]
        elif self.model_id == MODEL_QUAD3D:
            phi, th, psi = x[6], x[7], x[8]
            acc = p["a"] * u[0] + p["b"]
            cf, sf, ct, st, cp, sp = np.cos(phi), np.sin(phi), np.cos(th), np.sin(th), np.cos(psi), np.sin(psi)
            gx = cf * st * cp + sf * sp
            gy = cf * st * sp - sf * cp
            gz = cf * ct
            A[0, 1] = A[2, 3] = A[4, 5] = 1.0
            A[1, 6] = acc * (-sf * st * cp + cf * sp)
            A[1, 7] = acc * (cf * ct * cp)
            A[1, 8] = acc * (-cf * st * sp + sf * cp)
            B[1, 0] = p["a"] * gx
            A[3, 6] = acc * (-sf * st * sp - cf * cp)
            A[3, 7] = acc * (cf * ct * sp)
            A[3, 8] = acc * (cf * st * cp + sf * sp)
            B[3, 0] = p["a"] * gy
            A[5, 6] = acc * (-sf * ct)
            A[5, 7] = acc * (-cf * st)
            B[5, 0] = p["a"] * gz
            A[6, 9] = A[7, 10] = A[8, 11] = 1.0
            A[9, 6], A[9, 9], B[9, 1] = p["c"], p["d"], p["e"]
            A[10, 7], A[10, 10], B[10, 2] = p["f"], p["h"], p["l"]
            A[11, 8], A[11, 11], B[11, 3] = p["c"], p["d"], p["e"]
        elif self.model_id == MODEL_CARTPOLE:
            mc, mp, l = p["m_c"], p["m_p"], p["l"]
            M = mc + mp
            th, w, F = x[2], x[3], u[0]
            s, c = np.sin(th), np.cos(th)
            tmp = (F + mp * l * w * w * s) / M
            den = l * (4.0 / 3.0 - mp * c * c / M)
            num = g * s - c * tmp
            tha = num / den
            dtmp = np.array([mp * l * w * w * c / M, 2 * mp * l * w * s / M, 1.0 / M])  # th, w, F
            dden = np.array([l * 2 * mp * c * s / M, 0.0, 0.0])
            dnum = np.array([g * c + s * tmp - c * dtmp[0], -c * dtmp[1], -c * dtmp[2]])
            dtha = (dnum * den - num * dden) / den**2
            k = mp * l / M
            dxa = dtmp - k * (dtha * c - np.array([tha * s, 0.0, 0.0]))
            A[0, 1] = A[2, 3] = 1.0
            A[1, 2], A[1, 3], B[1, 0] = dxa
            A[3, 2], A[3, 3], B[3, 0] = dtha
        return A, B

    def prior_f(self, x: np.ndarray, u: np.ndarray, params: dict | None = None) -> np.ndarray:
        """Continuous-time prior dynamics f(x, u) for row-stacked states (n, nx) and inputs (n, nu)
        -- crazyflow's ``fc_func`` as used by `gpmpc/gpmpc.py:87,139,145,199` (``prior_dynamics``)."""
        p = self.prior if params is None else params
        x = np.atleast_2d(np.asarray(x, dtype=np.float64))
        u = np.atleast_2d(np.asarray(u, dtype=np.float64))
        f = np.zeros_like(x)
        g = self.gravity
        if self.model_id == MODEL_QUAD2D:
            th = x[:, 4]
            acc = p["a"] * u[:, 0] + p["b"]
            f[:, 0], f[:, 1], f[:, 2], f[:, 3] = x[:, 1], acc * np.sin(th), x[:, 3], acc * np.cos(th) - g
            f[:, 4], f[:, 5] = x[:, 5], p["f"] * th + p["h"] * x[:, 5] + p["l"] * u[:, 1]
        elif self.model_id == MODEL_QUAD3D:
            phi, th, psi = x[:, 6], x[:, 7], x[:, 8]
            acc = p["a"] * u[:, 0] + p["b"]
            cf, sf, ct, st, cp, sp = np.cos(phi), np.sin(phi), np.cos(th), np.sin(th), np.cos(psi), np.sin(psi)
            f[:, 0], f[:, 2], f[:, 4] = x[:, 1], x[:, 3], x[:, 5]
            f[:, 1] = acc * (cf * st * cp + sf * sp)
            f[:, 3] = acc * (cf * st * sp - sf * cp)
            f[:, 5] = acc * cf * ct - g
            f[:, 6], f[:, 7], f[:, 8] = x[:, 9], x[:, 10], x[:, 11]
            f[:, 9] = p["c"] * phi + p["d"] * x[:, 9] + p["e"] * u[:, 1]
            f[:, 10] = p["f"] * th + p["h"] * x[:, 10] + p["l"] * u[:, 2]
            f[:, 11] = p["c"] * psi + p["d"] * x[:, 11] + p["e"] * u[:, 3]
        elif self.model_id == MODEL_CARTPOLE:
            mc, mp, l = p["m_c"], p["m_p"], p["l"]
            M = mc + mp
            th, w, F = x[:, 2], x[:, 3], u[:, 0]
            s, c = np.sin(th), np.cos(th)
            tmp = (F + mp * l * w * w * s) / M
            tha = (g * s - c * tmp) / (l * (4.0 / 3.0 - mp * c * c / M))
            f[:, 0], f[:, 1], f[:, 2], f[:, 3] = x[:, 1], tmp - mp * l * tha * c / M, w, tha
        return f

    # ------------------------------------------------------------------ references
    def reference_trajectory(self, length: int | None = None) -> np.ndarray:
        """Periodic reference trajectory (nx, L).  The reference takes it from the
        crazyflow ``DroneFigureEightXY-v0`` env (`scripts/run_gp_mpc.py:150-151`), which is
        not installed; the build uses analytic figure-eights of the same kind."""
        L = self.traj_len if length is None else length
        t = np.arange(L) * self.dt
        w = 2 * np.pi / (L * self.dt)
        traj = np.zeros((self.nx, L))
        if self.model_id == MODEL_QUAD2D:
            traj[0] = np.sin(w * t)
            traj[1] = w * np.cos(w * t)
            traj[2] = 1.0 + 0.5 * np.sin(2 * w * t)
            traj[3] = w * np.cos(2 * w * t)
        elif self.model_id == MODEL_QUAD3D:
            traj[0] = np.sin(w * t)
            traj[1] = w * np.cos(w * t)
            traj[2] = 0.5 * np.sin(2 * w * t)
            traj[3] = w * np.cos(2 * w * t)
            traj[4] = 1.0
        elif self.model_id == MODEL_CARTPOLE:
            traj[0] = 0.5 * np.sin(w * t)
            traj[1] = 0.5 * w * np.cos(w * t)
        return traj

    def copy(self) -> "ModelSpec":
        """Independent copy (controllers apply their q_mpc / r_mpc / prior_params to a copy, so the
        caller's spec object is never mutated)."""
        return copy.deepcopy(self)

    def to_dict(self) -> dict:
        """Plain-number view of the spec (what the CPU oracle consumes)."""
        return dict(
            name=self.name, nx=self.nx, nu=self.nu, dt=self.dt, gravity=self.gravity,
            prior=dict(self.prior), u_eq=self.u_eq.copy(), x_lo=self.x_lo.copy(), x_hi=self.x_hi.copy(),
            u_lo=self.u_lo.copy(), u_hi=self.u_hi.copy(), q_diag=self.q_diag.copy(), r_diag=self.r_diag.copy(),
            gp_inputs=[list(i) for i in self.gp_inputs], var_inputs=[list(i) for i in self.var_inputs],
            unc_dims=list(self.unc_dims),
        )


_Q3 = np.array([8, 0.1, 8, 0.1, 8, 0.1, 0.5, 0.5, 0.5, 0.001, 0.001, 0.001])  # gp_mpc_config.yaml:7
_R3 = np.array([3, 3, 3, 0.1])                                                 # gp_mpc_config.yaml:8
_XLO3 = np.array([-2, -15, -2, -15, -0.05, -15, -1.5, -1.5, -10, -8.5, -8.5, -10.0])  # gpmpc.py:242
_XHI3 = np.array([2, 15, 2, 15, 2, 15, 1.5, 1.5, 10, 8.5, 8.5, 10.0])                  # gpmpc.py:243
_ULO3 = np.array([0.12, -0.43, -0.43, -0.43])                                          # gpmpc.py:245
_UHI3 = np.array([0.59, 0.43, 0.43, 0.43])                                             # gpmpc.py:246


def quad3d_spec() -> ModelSpec:
    nx = 12
    return ModelSpec(
        name="quad3d", model_id=MODEL_QUAD3D, nx=nx, nu=4, dt=0.02,
        prior=dict(REF_PRIOR), true_params=dict(TRUE_QUAD),
        u_eq=np.array([0.3234, 0, 0, 0.0]),                    # gpmpc.py:18
        x_lo=_XLO3.copy(), x_hi=_XHI3.copy(), u_lo=_ULO3.copy(), u_hi=_UHI3.copy(),
        q_diag=_Q3.copy(), r_diag=_R3.copy(),
        # idx_T, idx_R, idx_P over z = [x; u]   (gpmpc.py:173)
        gp_inputs=((nx + 0,), (6, 9, nx + 1), (7, 10, nx + 2)),
        # the reference evaluates the variance at z[:, gp_idx] with gp_idx indexing the
        # 7-dim GP-input space (gpmpc.py:59 vs :437-444) -- reproduced.
        var_inputs=((0,), (1, 2, 3), (4, 5, 6)),
        unc_dims=(1, 3, 5, 9, 10),                               # gpmpc.py:68
        gp_names=("T", "R", "P"),
    )


def quad2d_spec() -> ModelSpec:
    nx = 6
    sel_x = [0, 1, 4, 5, 7, 10]  # x, vx, z, vz, theta, dtheta of the 3D state
    sel_u = [0, 2]               # T_c, P_c
    return ModelSpec(
        name="quad2d", model_id=MODEL_QUAD2D, nx=nx, nu=2, dt=0.02,
        prior=dict(REF_PRIOR), true_params=dict(TRUE_QUAD),
        u_eq=np.array([0.3234, 0.0]),
        x_lo=_XLO3[sel_x].copy(), x_hi=_XHI3[sel_x].copy(),
        u_lo=_ULO3[sel_u].copy(), u_hi=_UHI3[sel_u].copy(),
        q_diag=_Q3[sel_x].copy(), r_diag=_R3[sel_u].copy(),
        gp_inputs=((nx + 0,), (4, 5, nx + 1)),
        var_inputs=((nx + 0,), (4, 5, nx + 1)),
        unc_dims=(1, 3, 5),
        gp_names=("T", "P"),
    )


def cartpole_spec() -> ModelSpec:
    nx = 4
    prior = dict(m_c=1.0, m_p=0.1, l=0.5)
    true = dict(m_c=1.2, m_p=0.12, l=0.55)
    return ModelSpec(
        # dt = 0.05 s: at H = 20 the horizon spans 1 s.  With dt = 0.02 (0.4 s) the
        # terminal cost W_e = Q (the reference's convention, gpmpc.py:231-239) does not
        # stabilise the inverted pole: even the nominal closed loop drifted off the
        # reference and the GP loop ran into the SQP iteration limit (CPU restatement
        # and GPU kernel alike).
        name="cartpole", model_id=MODEL_CARTPOLE, nx=nx, nu=1, dt=0.05,
        prior=prior, true_params=true,
        u_eq=np.array([0.0]),
        x_lo=np.array([-5.0, -10.0, -1.0, -10.0]), x_hi=np.array([5.0, 10.0, 1.0, 10.0]),
        u_lo=np.array([-10.0]), u_hi=np.array([10.0]),
        q_diag=np.array([1.0, 0.1, 1.0, 0.1]), r_diag=np.array([0.1]),
        gp_inputs=((2, 3, nx), (2, 3, nx)),
        var_inputs=((2, 3, nx), (2, 3, nx)),
        unc_dims=(1, 3),
        gp_names=("x_acc", "theta_acc"),
    )


SPECS = {"quad2d": quad2d_spec, "quad3d": quad3d_spec, "cartpole": cartpole_spec}


def get_spec(name: str) -> ModelSpec:
    try:
        return SPECS[name]()
    except KeyError:
        raise ValueError(f"unknown model {name!r}; expected one of {sorted(SPECS)}") from None
