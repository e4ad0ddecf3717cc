"""ORACLE — test infrastructure only (see ba_oracle.cpp header).

ctypes wrapper around liboracle.so, the C++ CPU restatement of the
reference's Ceres LM + DENSE_SCHUR bundle adjustment.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
PARITY UNPINNED with respect to the reference itself (no reference fixtures
exist and Ceres is not available): see DESIGN.md §5.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
LOG_FIELDS = ["iteration", "cost", "cost_change", "gradient_max_norm", "gradient_norm", "step_norm",
              "relative_decrease", "trust_region_radius", "step_is_valid", "step_is_successful",
              "model_cost_change", "linear_solver_iterations"]
TERMINATION = {0: "CONVERGENCE", 1: "NO_CONVERGENCE", 2: "FAILURE"}


class _Problem(C.Structure):
    _fields_ = [("n_cams", C.c_int32), ("n_pts", C.c_int32), ("n_obs", C.c_int32), ("pad", C.c_int32),
                ("cams", C.c_void_p), ("cam_fixed", C.c_void_p), ("cam_fixed_extr", C.c_void_p), ("K", C.c_void_p),
                ("pts", C.c_void_p), ("pt_fixed", C.c_void_p), ("obs_cam", C.c_void_p), ("obs_pt", C.c_void_p),
                ("obs_uv", C.c_void_p), ("huber_a", C.c_double)]


class Options(C.Structure):
    _fields_ = [("max_num_iterations", C.c_int32), ("max_num_consecutive_invalid_steps", C.c_int32),
                ("jacobi_scaling", C.c_int32), ("linear_solver", C.c_int32),
                ("function_tolerance", C.c_double), ("gradient_tolerance", C.c_double),
                ("parameter_tolerance", C.c_double), ("initial_trust_region_radius", C.c_double),
                ("max_trust_region_radius", C.c_double), ("min_trust_region_radius", C.c_double),
                ("min_relative_decrease", C.c_double), ("min_lm_diagonal", C.c_double),
                ("max_lm_diagonal", C.c_double),
                # ITERATIVE_SCHUR (ceres defaults: JACOBI, 500, 0, fp64, eta 0.1)
                ("preconditioner_type", C.c_int32), ("max_linear_solver_iterations", C.c_int32),
                ("min_linear_solver_iterations", C.c_int32), ("precision", C.c_int32), ("eta", C.c_double)]


def build(force: bool = False) -> Path:
    src = HERE / "ba_oracle.cpp"
    if force or not LIB.exists() or LIB.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["make", "-C", str(HERE), "-s"], check=True)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        L.oracle_solve.restype = C.c_int
        L.oracle_solve.argtypes = [C.POINTER(_Problem), C.POINTER(Options), C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_linearize.restype = C.c_int
        L.oracle_linearize.argtypes = [C.POINTER(_Problem), C.c_void_p, C.c_void_p, C.POINTER(C.c_double)]
        L.oracle_residuals.argtypes = [C.POINTER(_Problem), C.c_void_p]
        for f in ("oracle_angle_axis_to_R", "oracle_R_to_angle_axis"):
            getattr(L, f).argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_angle_axis_to_R_jac.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_default_options.argtypes = [C.POINTER(Options)]
        L.oracle_set_threads.argtypes = [C.c_int]
        L.oracle_bench.restype = C.c_double
        L.oracle_bench.argtypes = [C.POINTER(_Problem), C.c_int, C.c_double]
        L.oracle_max_threads.restype = C.c_int
        L.oracle_prune.argtypes = [C.c_int] + [C.c_void_p] * 9
        L.oracle_camera_colnorm2.argtypes = [C.POINTER(_Problem), C.c_void_p]
        L.oracle_reduced_system.restype = C.c_int
        L.oracle_reduced_system.argtypes = [C.POINTER(_Problem), C.c_void_p, C.c_double, C.c_int, C.c_void_p,
                                            C.c_void_p]
        _lib = L
    return _lib


def default_options(**kw) -> Options:
    o = Options()
    lib().oracle_default_options(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _make(problem, cams, pts):
    s = _Problem()
    s.n_cams, s.n_pts, s.n_obs = problem.n_cams, problem.n_pts, problem.n_obs
    s.cams, s.pts = _p(cams), _p(pts)
    s.cam_fixed, s.cam_fixed_extr, s.K = _p(problem.cam_fixed), _p(problem.cam_fixed_extr), _p(problem.K)
    s.pt_fixed, s.obs_cam, s.obs_pt, s.obs_uv = (_p(problem.pt_fixed), _p(problem.obs_cam), _p(problem.obs_pt),
                                                _p(problem.obs_uv))
    s.huber_a = problem.huber_a
    return s


def set_threads(n: int):
    lib().oracle_set_threads(int(n))


def max_threads() -> int:
    return int(lib().oracle_max_threads())


def bench_seconds_per_iteration(problem, iters: int = 2, radius: float = 1e4) -> float:
    """CPU baseline: seconds per LM iteration (linearise + Schur + solve +
    candidate), the same work as the GPU bench step."""
    p = problem.normalized()
    cams, pts = p.cams.copy(), p.pts.copy()
    s = _make(p, cams, pts)
    return float(lib().oracle_bench(C.byref(s), int(iters), float(radius)))


def solve(problem, options: Options | None = None, max_log: int = 1024):
    """Returns (cams, pts, summary dict, iteration log list)."""
    p = problem.normalized()
    cams = p.cams.copy()
    pts = p.pts.copy()
    s = _make(p, cams, pts)
    o = options or default_options()
    log = np.zeros((max_log, 12))
    summ = np.zeros(6)
    n = lib().oracle_solve(C.byref(s), C.byref(o), _p(log), max_log, _p(summ))
    recs = [dict(zip(LOG_FIELDS, row)) for row in log[:min(n, max_log)]]
    for r in recs:
        for k in ("iteration", "step_is_valid", "step_is_successful", "linear_solver_iterations"):
            r[k] = int(r[k])
    summary = dict(initial_cost=summ[0], final_cost=summ[1], num_iterations=int(summ[2]),
                   num_successful_steps=int(summ[3]), num_unsuccessful_steps=int(summ[4]),
                   termination_type=TERMINATION[int(summ[5])])
    return cams, pts, summary, recs


def linearize(problem):
    p = problem.normalized()
    s = _make(p, p.cams, p.pts)
    r = np.empty((p.n_obs, 2))
    J = np.empty((p.n_obs, 2, 9))
    cost = C.c_double()
    rc = lib().oracle_linearize(C.byref(s), _p(r), _p(J), C.byref(cost))
    return r, J, cost.value, rc == 0


def residuals(problem):
    p = problem.normalized()
    s = _make(p, p.cams, p.pts)
    r = np.empty((p.n_obs, 2))
    lib().oracle_residuals(C.byref(s), _p(r))
    return r


def angle_axis_to_R(w):
    w = np.ascontiguousarray(w, np.float64)
    R = np.empty(9)
    lib().oracle_angle_axis_to_R(_p(w), _p(R))
    return R.reshape(3, 3).T  # column-major -> [row, col]


def angle_axis_to_R_jac(w):
    w = np.ascontiguousarray(w, np.float64)
    R = np.empty(9)
    dR = np.empty(27)
    lib().oracle_angle_axis_to_R_jac(_p(w), _p(R), _p(dR))
    return R.reshape(3, 3).T, dR.reshape(3, 3, 3).transpose(0, 2, 1)


def R_to_angle_axis(R):
    Rc = np.ascontiguousarray(np.asarray(R, np.float64).T.reshape(9))
    w = np.empty(3)
    lib().oracle_R_to_angle_axis(_p(Rc), _p(w))
    return w


def prune(extr, cam_center, K, obs_cam, obs_X, obs_uv, obs_inv_sigma, obs_dist):
    """pruneCorrespondences restated (Optimizer.cpp:6-79), float; returns uint8
    codes 0 inlier, 1 behind, 2 depth range, 3 chi test (see ba_prune)."""
    f32 = [np.ascontiguousarray(a, dtype=np.float32) for a in (extr, cam_center, K)]
    oc = np.ascontiguousarray(obs_cam, dtype=np.int32)
    o32 = [np.ascontiguousarray(a, dtype=np.float32) for a in (obs_X, obs_uv, obs_inv_sigma, obs_dist)]
    out = np.empty(oc.size, np.uint8)
    lib().oracle_prune(int(oc.size), *[_p(a) for a in f32], _p(oc), *[_p(a) for a in o32], _p(out))
    return out


def camera_colnorm2(problem):
    """Camera column norms^2 of the corrected jacobian [n_cams, 6] (additive
    over point shards)."""
    cams, pts = problem.cams.copy(), problem.pts.copy()
    s = _make(problem, cams, pts)
    out = np.zeros((problem.n_cams, 6))
    lib().oracle_camera_colnorm2(C.byref(s), _p(out))
    return out


def reduced_system(problem, radius=1e4, cam_colnorm2=None, add_cam_D=True):
    """Reduced camera system (lower triangle, rhs) of one LM step at iteration-0
    scaling; cam_colnorm2: global camera column norms for a point shard."""
    cams, pts = problem.cams.copy(), problem.pts.copy()
    s = _make(problem, cams, pts)
    nmax = 6 * problem.n_cams
    lhs = np.zeros((nmax, nmax))
    rhs = np.zeros(nmax)
    cn = None if cam_colnorm2 is None else np.ascontiguousarray(cam_colnorm2, dtype=np.float64)
    n = lib().oracle_reduced_system(C.byref(s), _p(cn), float(radius), int(bool(add_cam_D)), _p(lhs), _p(rhs))
    if n < 0:
        raise RuntimeError("oracle_reduced_system failed")
    return lhs.reshape(-1)[: n * n].reshape(n, n).copy(), rhs[:n].copy()
