"""ctypes binding of the C++ CPU restatement (oracle/cpu_ref.cpp) -- TEST / BASELINE ONLY.

Loaded by tests/ (parity of the C++ restatement against the numpy oracle) and by bench.py's
``cpu_baseline`` leg (the timed CPU path, OpenMP over instances).  Build: ``make -C oracle``.
"""

from __future__ import annotations

import ctypes
from pathlib import Path

import numpy as np

import os

# CPUREF_LIB: another build of the same source (the sanitizer build of tools/asan_cpu_ref.sh)
LIB_PATH = Path(os.environ.get("CPUREF_LIB", Path(__file__).resolve().parent / "lib" / "libcpuref.so"))
_P, _I, _D = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
_SIGS = {
    "cpuref_create": (_P, [_I, _I, _P, _I, _D, _P, _P, _P, _P, _P, _P, _P, _D, _I]),
    "cpuref_destroy": (None, [_P]),
    "cpuref_set_options": (None, [_P, _I, _D, _I, _D]),
    "cpuref_set_gp": (_I, [_P, _I, _I, _I, _P, _P, _P, _D, _D, _D, _P, _P]),
    "cpuref_set_gp_var": (_I, [_P, _I, _I, _P, _P]),
    "cpuref_set_gp_var_root": (_I, [_P, _I, _I, _I, _P]),
    "cpuref_gp_var": (_I, [_P, _I, _I, _P, _P]),
    "cpuref_use_gp": (None, [_P, _I]),
    "cpuref_set_tightening": (None, [_P, _I, _D, _P, _P, _P, _P, _I]),
    "cpuref_set_reference": (None, [_P, _P, _I]),
    "cpuref_step": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I]),
}
_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle`")
        lib = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib = lib
    return _lib


def _c(a, dtype=np.float64):
    return np.ascontiguousarray(a, dtype=dtype)


class CpuRef:
    """B instances of the control step on the host (GPMPC.select_action semantics, batched)."""

    def __init__(self, spec, H: int, B: int, gps=None, lqr_mats=None, prob: float = 0.95, uh: float = -1e-8,
                 tol: float = 1e-6, qp_tol: float | None = None, qp_max_iter: int = 50, max_iter: int = 25, fitc=None,
                 love_roots=None):
        """``fitc[g] = (S (M, d), w (M,))``: GP g's mean over the inducing rows S with weights w
        (`gpmpc/gpmpc.py:175-187,377-400`); its variance stays the exact GP's (``gps[g]``).
        ``love_roots[g]`` (n, r) or None: GP g's tightening variance from that LOVE root (the
        reference's ``fast_pred_var``, `gpmpc/gpmpc.py:442-444`) instead of the exact L^-1 k."""
        from oracle import gpmpc_oracle as O

        self.lib = load()
        self.spec, self.H, self.B = spec, H, B
        nx, nu = spec.nx, spec.nu
        self._keep = [_c(spec.param_vector()), _c(spec.x_lo), _c(spec.x_hi), _c(spec.u_lo), _c(spec.u_hi),
                      _c(spec.q_diag), _c(spec.r_diag), _c(spec.u_eq)]
        k = self._keep
        self.h = self.lib.cpuref_create(spec.model_id, H, k[0].ctypes.data, len(k[0]), spec.dt, k[1].ctypes.data,
                                        k[2].ctypes.data, k[3].ctypes.data, k[4].ctypes.data, k[5].ctypes.data,
                                        k[6].ctypes.data, k[7].ctypes.data, uh, 1)
        if not self.h:
            raise RuntimeError("cpuref_create failed")
        # qp_tol None: the NLP tolerance (acados passes its NLP tolerances on to the QP solver)
        self.lib.cpuref_set_options(self.h, max_iter, tol, qp_max_iter, tol if qp_tol is None else qp_tol)
        traj = _c(spec.reference_trajectory().T)
        self._keep.append(traj)
        self.lib.cpuref_set_reference(self.h, traj.ctypes.data, traj.shape[0])
        if gps is not None:
            for g, gp in enumerate(gps):
                X, a, L = _c(gp.X), _c(gp.alpha), _c(gp.L)
                ii = _c(spec.gp_inputs[g], np.int32)
                vi = _c(spec.var_inputs[g], np.int32)
                self._keep += [X, a, L, ii, vi]
                if fitc is not None and fitc[g] is not None:
                    S, w = _c(fitc[g][0]), _c(fitc[g][1])
                    self._keep += [S, w]
                    rc = self.lib.cpuref_set_gp(self.h, g, S.shape[0], S.shape[1], S.ctypes.data, w.ctypes.data,
                                                None, gp.ell, gp.sf2, gp.sn2, ii.ctypes.data, vi.ctypes.data)
                    rc = rc or self.lib.cpuref_set_gp_var(self.h, g, X.shape[0], X.ctypes.data, L.ctypes.data)
                else:
                    rc = self.lib.cpuref_set_gp(self.h, g, X.shape[0], X.shape[1], X.ctypes.data, a.ctypes.data,
                                                L.ctypes.data, gp.ell, gp.sf2, gp.sn2, ii.ctypes.data, vi.ctypes.data)
                if rc == 0 and love_roots is not None and love_roots[g] is not None:
                    R = _c(love_roots[g])
                    self._keep.append(R)
                    rc = self.lib.cpuref_set_gp_var_root(self.h, g, R.shape[0], R.shape[1], R.ctypes.data)
                if rc != 0:
                    raise RuntimeError(f"cpuref_set_gp({g}) failed")
            self.lib.cpuref_use_gp(self.h, 1)
        if lqr_mats is not None:
            Ad, Bd, K = (_c(m) for m in lqr_mats)
            unc = _c(spec.unc_dims, np.int32)
            self._keep += [Ad, Bd, K, unc]
            self.lib.cpuref_set_tightening(self.h, 1, O.inverse_cdf(prob, nx), Ad.ctypes.data, Bd.ctypes.data,
                                           K.ctypes.data, unc.ctypes.data, len(unc))
        n = H * (nx + nu)
        self.x = np.zeros((B, H + 1, nx))
        self.u = np.zeros((B, H, nu))
        self.pi = np.zeros((B, H, nx))
        self.ll = np.zeros((B, n))
        self.lu = np.zeros((B, n))
        self.has_prev = np.zeros(B, np.int32)
        self.u0 = np.zeros((B, nu))
        self.status = np.zeros(B, np.int32)
        self.sqp_iter = np.zeros(B, np.int32)
        self.qp_iter = np.zeros(B, np.int32)

    def gp_var(self, g: int, Z: np.ndarray) -> np.ndarray:
        """GP g's tightening variance (noise included) at Z (P, d): exact or from its LOVE root."""
        Z = _c(Z)
        out = np.zeros(Z.shape[0])
        if self.lib.cpuref_gp_var(self.h, g, Z.shape[0], Z.ctypes.data, out.ctypes.data) != 0:
            raise RuntimeError(f"cpuref_gp_var({g}) failed")
        return out

    def step(self, x0: np.ndarray, tstep: np.ndarray, threads: int = 1) -> np.ndarray:
        x0 = _c(x0)
        ts = _c(tstep, np.int32)
        a = [x0, ts, self.x, self.u, self.pi, self.ll, self.lu, self.has_prev, self.u0, self.status, self.sqp_iter,
             self.qp_iter]
        self.lib.cpuref_step(self.h, self.B, *[v.ctypes.data for v in a], threads)
        return self.u0

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.cpuref_destroy(self.h)
            self.h = None
