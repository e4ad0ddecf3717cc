"""ctypes binding of libba_hip.so (include/ba_hip.h).

The product path has no CPU fallback: if the HIP library is missing or fails
to load, every entry point raises ``NativeLibraryError``.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "libba_hip.so"

BA_OK = 0
BA_ABI_VERSION = 2          # include/ba_hip.h
STATUS_NAMES = {0: "BA_OK", 1: "BA_ERR_INVALID_ARGUMENT", 2: "BA_ERR_DEVICE", 3: "BA_ERR_OUT_OF_MEMORY",
                4: "BA_ERR_NO_PROBLEM", 5: "BA_ERR_COMM"}
TERMINATION_NAMES = {0: "CONVERGENCE", 1: "NO_CONVERGENCE", 2: "FAILURE"}


class NativeLibraryError(RuntimeError):
    pass


class BAError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class ba_problem(C.Structure):
    _fields_ = [
        ("n_cams", C.c_int32), ("n_pts", C.c_int32), ("n_obs", C.c_int32), ("reserved", C.c_int32),
        ("cams", C.c_void_p), ("cam_fixed", C.c_void_p), ("cam_fixed_extr", C.c_void_p), ("K", C.c_void_p),
        ("pts", C.c_void_p), ("pt_fixed", C.c_void_p), ("obs_cam", C.c_void_p), ("obs_pt", C.c_void_p),
        ("obs_uv", C.c_void_p), ("huber_a", C.c_double),
    ]


class ba_options(C.Structure):
    _fields_ = [
        ("max_num_iterations", C.c_int32), ("max_num_consecutive_invalid_steps", C.c_int32),
        ("jacobi_scaling", C.c_int32), ("linear_solver", C.c_int32),
        ("function_tolerance", C.c_double), ("gradient_tolerance", C.c_double),
        ("parameter_tolerance", C.c_double), ("initial_trust_region_radius", C.c_double),
        ("max_trust_region_radius", C.c_double), ("min_trust_region_radius", C.c_double),
        ("min_relative_decrease", C.c_double), ("min_lm_diagonal", C.c_double), ("max_lm_diagonal", C.c_double),
        ("preconditioner_type", C.c_int32), ("max_linear_solver_iterations", C.c_int32),
        ("min_linear_solver_iterations", C.c_int32), ("precision", C.c_int32), ("eta", C.c_double),
    ]


class ba_summary(C.Structure):
    _fields_ = [
        ("initial_cost", C.c_double), ("final_cost", C.c_double), ("num_iterations", C.c_int32),
        ("num_successful_steps", C.c_int32), ("num_unsuccessful_steps", C.c_int32),
        ("termination_type", C.c_int32), ("total_time_s", C.c_double), ("linearize_time_s", C.c_double),
        ("solve_time_s", C.c_double),
    ]


class ba_iteration(C.Structure):
    _fields_ = [
        ("iteration", C.c_int32), ("step_is_valid", C.c_int32), ("step_is_successful", C.c_int32),
        ("linear_solver_iterations", C.c_int32), ("cost", C.c_double), ("cost_change", C.c_double),
        ("gradient_max_norm", C.c_double), ("gradient_norm", C.c_double), ("step_norm", C.c_double),
        ("relative_decrease", C.c_double), ("trust_region_radius", C.c_double),
        ("model_cost_change", C.c_double), ("iteration_time_s", C.c_double),
    ]


class ba_prune_problem(C.Structure):
    _fields_ = [
        ("n_cams", C.c_int32), ("n_obs", C.c_int32),
        ("extr", C.c_void_p), ("cam_center", C.c_void_p), ("K", C.c_void_p), ("obs_cam", C.c_void_p),
        ("obs_X", C.c_void_p), ("obs_uv", C.c_void_p), ("obs_inv_sigma", C.c_void_p), ("obs_dist", C.c_void_p),
    ]


class ba_pose_batch(C.Structure):
    _fields_ = [
        ("n_problems", C.c_int32), ("reserved", C.c_int32), ("obs_offset", C.c_void_p), ("cams", C.c_void_p),
        ("K", C.c_void_p), ("pts", C.c_void_p), ("obs_uv", C.c_void_p), ("huber_a", C.c_double),
    ]


# int (*)(void* user, double* values, int64_t n, int op) of ba_comm_init_host
HOST_ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int64, C.c_int)

PRUNE_NAMES = {0: "INLIER", 1: "OUTLIER_BEHIND", 2: "OUTLIER_DEPTH", 3: "OUTLIER_CHI2"}


# (name, restype, argtypes) — every symbol declared in include/ba_hip.h
SIGNATURES = [
    ("ba_abi_version", C.c_int, []),
    ("ba_default_options", None, [C.POINTER(ba_options)]),
    ("ba_create", C.c_int, [C.POINTER(C.c_void_p), C.c_int]),
    ("ba_destroy", C.c_int, [C.c_void_p]),
    ("ba_last_error", C.c_char_p, [C.c_void_p]),
    ("ba_comm_unique_id", C.c_int, [C.c_char_p]),
    ("ba_comm_init", C.c_int, [C.c_void_p, C.c_char_p, C.c_int, C.c_int]),
    ("ba_comm_allreduce_host", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
    ("ba_comm_init_host", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
    ("ba_set_problem", C.c_int, [C.c_void_p, C.POINTER(ba_problem)]),
    ("ba_set_params", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("ba_solve", C.c_int, [C.c_void_p, C.POINTER(ba_options), C.POINTER(ba_summary)]),
    ("ba_get_params", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("ba_get_iteration_log", C.c_int, [C.c_void_p, C.POINTER(ba_iteration), C.c_int]),
    ("ba_eval_residuals", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_double)]),
    ("ba_linearize", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_double)]),
    ("ba_bench_iteration_times", C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    ("ba_debug_blocks", C.c_int, [C.c_void_p, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]),
    ("ba_prune", C.c_int, [C.c_void_p, C.POINTER(ba_prune_problem), C.c_void_p]),
    ("ba_solve_pose_batch", C.c_int, [C.c_void_p, C.POINTER(ba_pose_batch), C.POINTER(ba_options), C.c_void_p,
                                      C.POINTER(ba_summary)]),
    ("ba_synchronize", C.c_int, [C.c_void_p]),
    ("ba_bench_iterations", C.c_int, [C.c_void_p, C.POINTER(ba_options), C.c_int, C.c_double,
                                      C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    ("ba_stream_copy", C.c_int, [C.c_void_p, C.c_size_t, C.c_int, C.POINTER(C.c_double)]),
]

_LIB = None


def load_library(path: str | os.PathLike | None = None):
    """Load libba_hip.so (in-tree).  Raises NativeLibraryError if absent."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    # BA_HIP_LIB: load another build of the same ABI (A/B kernel comparisons)
    p = Path(path) if path else Path(os.environ.get("BA_HIP_LIB", str(LIB_PATH)))
    if not p.exists():
        raise NativeLibraryError(
            f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            f"(hipcc --offload-arch=gfx950).  There is no CPU fallback.")
    try:
        lib = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - environment specific
        raise NativeLibraryError(f"failed to load {p}: {e}") from e
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.ba_abi_version() != BA_ABI_VERSION:
        raise NativeLibraryError("ABI version mismatch")
    if path is None:
        _LIB = lib
    return lib


def default_options() -> ba_options:
    o = ba_options()
    load_library().ba_default_options(C.byref(o))
    return o
