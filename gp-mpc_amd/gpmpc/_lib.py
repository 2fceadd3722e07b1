"""ctypes binding of the C ABI in ``include/gpmpc_mi355x.h`` (libgpmpc_mi355x.so).

The product path has no CPU fallback: if the HIP library is missing or no GPU is present,
every entry point raises :class:`GPMPCError`.  torch is imported first so that the library
binds to the same HIP runtime instance torch uses (same ``libamdhip64.so.7`` soname) and
torch device pointers / streams are valid on both sides.
"""

from __future__ import annotations

import ctypes
import hashlib
import os
from ctypes import POINTER, c_char_p, c_double, c_int32, c_int64, c_void_p
from pathlib import Path

import torch  # noqa: F401  (HIP runtime shared with torch)

_DEFAULT_LIB = Path(__file__).resolve().parent / "lib" / "libgpmpc_mi355x.so"
LIB_PATH = Path(os.environ.get("GPMPC_LIB", _DEFAULT_LIB))
CSRC = Path(__file__).resolve().parents[1] / "csrc"
# the files gpmpc_build_id's source hash covers, in the Makefile's order (HASHED)
HASHED = ["sqp_kernel.hip", "gp_kernels.hip", "capi.hip", "gpmpc_common.h", "models.h",
          "../../include/gpmpc_mi355x.h", "build_id.cpp", "Makefile"]

_lib = None

# C-ABI symbols and their signatures (restype, argtypes).
_D = c_double
_I = c_int32
_P = c_void_p
SIGNATURES = {
    "gpmpc_create": (_I, [_I, _I, _I, _I, POINTER(_P)]),
    "gpmpc_destroy": (None, [_P]),
    "gpmpc_last_error": (c_char_p, []),
    "gpmpc_set_model": (_I, [_P, _P, _I, _D, _P, _P, _P, _P, _P, _P, _P, _D, _I]),
    "gpmpc_set_reference": (_I, [_P, _P, _I]),
    "gpmpc_set_options": (_I, [_P, _I, _D, _D, _D, _D, _I, _D, _D]),
    "gpmpc_set_gp": (_I, [_P, _I, _I, _I, _P, _P, _I, _P, _P, _D, _D, _D]),
    "gpmpc_use_gp": (_I, [_P, _I]),
    "gpmpc_set_gp_variance_root": (_I, [_P, _I, _I, _I, _P]),
    "gpmpc_set_tightening": (_I, [_P, _I, _D, _P, _P, _P]),
    "gpmpc_set_var_inputs": (_I, [_P, _I, _P, _I]),
    "gpmpc_reset": (_I, [_P, _I, _I, _P]),
    "gpmpc_set_iterate": (_I, [_P, _I, _P, _P, _P]),
    "gpmpc_solve": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "gpmpc_get_solution": (_I, [_P, _I, _P, _P, _P, _P]),
    "gpmpc_gp_predict": (_I, [_P, _I, _P, _I, _P, _P, _I, _P]),
    "gpmpc_gp_mean_grad": (_I, [_P, _I, _P, _I, _P, _P, _P]),
    "gpmpc_gp_posterior": (_I, [_I, _I, _I, _P, _P, _D, _D, _D, _P, _I, _P, _P, _I, _P]),
    "gpmpc_plant_step": (_I, [_P, _I, _P, _P, _P, _P, _P, _P]),
    "gpmpc_set_launch": (_I, [_P, _I]),
    "gpmpc_set_profiling": (_I, [_P, _I]),
    "gpmpc_kernel_times": (_I, [_P, POINTER(_D), POINTER(_I), POINTER(_D), POINTER(_I)]),
    "gpmpc_kernel_time_list": (_I, [_P, _I, _P, _P, _P, _P]),
    "gpmpc_set_timing_buffer": (_I, [_P, _P]),
    "gpmpc_set_stats_buffer": (_I, [_P, _P, _I]),
    "gpmpc_get_variance": (_I, [_P, _I, _P, _P]),
    "gpmpc_lds_bytes": (c_int64, [_I, _I]),
    "gpmpc_get_launch_info": (_I, [_P, _I, POINTER(_I), POINTER(_I)]),
    "gpmpc_get_launch_segments": (_I, [_P, _I, POINTER(_I)]),
    "gpmpc_set_tuning": (_I, [_P, _I, _I]),
    "gpmpc_set_cost_buffer": (_I, [_P, _P]),
    "gpmpc_build_id": (c_char_p, []),
}

# gpmpc_set_tuning options (include/gpmpc_mi355x.h GPMPC_TUNE_*)
TUNE = {"lin_cache": 0, "order": 1, "overlap": 2, "var_split": 3, "event_fence": 4, "seg": 5, "tail": 6, "seg_pivot": 7}


class GPMPCError(RuntimeError):
    pass


def source_hash() -> str:
    """sha256 (16 hex digits) of the library's sources in this tree, as the Makefile embeds it."""
    h = hashlib.sha256()
    for name in HASHED:
        h.update((CSRC / name).read_bytes())
    return h.hexdigest()[:16]


def build_id() -> str:
    """gpmpc_build_id() of the loaded library: 'src=<hash> git=<commit>[+dirty] kind=<product|timing>'."""
    return load(require_gpu=False).gpmpc_build_id().decode()


def build_info() -> dict:
    """The loaded library's build id, the tree's source hash and whether they match."""
    bid = build_id()
    src = bid.split()[0][4:] if bid.startswith("src=") else None
    tree = source_hash()
    return {"build_id": bid, "lib": str(LIB_PATH), "src_hash_lib": src, "src_hash_tree": tree,
            "matches_tree": src == tree}


def load(require_gpu: bool = True):
    """Load the HIP library (raises GPMPCError if it is missing; optionally if no GPU).

    The in-tree library must have been built from the sources next to it: its embedded source hash
    (gpmpc_build_id) is checked against the tree, so a stale library -- or an A/B variant left in its
    place -- fails loudly instead of running silently.  A library chosen by GPMPC_LIB (tools' A/B
    builds) is not checked."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise GPMPCError(f"HIP extension not built: {LIB_PATH} is missing (run __graft_entry__.build())")
        lib = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if LIB_PATH.resolve() == _DEFAULT_LIB.resolve() and (CSRC / "Makefile").exists():
            bid = lib.gpmpc_build_id().decode()
            want = source_hash()
            if f"src={want} " not in bid + " ":
                raise GPMPCError(f"stale HIP library {LIB_PATH}: built from sources {bid}, the tree has src={want} "
                                 "(rebuild: make -C gp-mpc_amd/csrc)")
        _lib = lib
    if require_gpu and not torch.cuda.is_available():
        raise GPMPCError("no HIP device available: the GP-MPC path runs only on the GPU (no CPU fallback)")
    return _lib


def check(status: int) -> None:
    if status != 0:
        msg = _lib.gpmpc_last_error().decode() if _lib is not None else "library not loaded"
        raise GPMPCError(f"gpmpc C-ABI error {status}: {msg}")


def ptr(t) -> int | None:
    """Raw pointer of a tensor / numpy array (None passes NULL)."""
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        return t.data_ptr()
    return t.ctypes.data


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
