"""Host-side Python handle on libba_hip.so: one `Solver` per (process, GPU).

Mirrors the ceres::Problem / ceres::Solve seam the reference uses
(ba_project/src/ba/Optimizer.cpp:225-242): build the problem, solve with the
options of BAOptimizer::configureSolver (Optimizer.cpp:80-90), read back the
parameters.  Everything numeric runs in the HIP library.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native as N
from .problem import HUBER_A, Problem


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


@dataclass
class Options:
    """ceres::Solver::Options fields used by the reference (+ Ceres defaults)."""
    max_num_iterations: int = 50
    max_num_consecutive_invalid_steps: int = 5
    jacobi_scaling: bool = True
    function_tolerance: float = 1e-6
    gradient_tolerance: float = 1e-10
    parameter_tolerance: float = 1e-8
    initial_trust_region_radius: float = 1e4
    max_trust_region_radius: float = 1e16
    min_trust_region_radius: float = 1e-32
    min_relative_decrease: float = 1e-3
    min_lm_diagonal: float = 1e-6
    max_lm_diagonal: float = 1e32
    # linear solver: "DENSE_SCHUR" (the reference's, Optimizer.cpp:85) or
    # "ITERATIVE_SCHUR" (implicit Schur + PCG, for C5-scale camera counts)
    linear_solver_type: str = "DENSE_SCHUR"
    preconditioner_type: str = "JACOBI"        # ceres default; or "SCHUR_JACOBI"
    max_linear_solver_iterations: int = 500
    min_linear_solver_iterations: int = 0
    eta: float = 1e-1
    precision: str = "FP64"                    # or "MIXED_FP32" (ITERATIVE_SCHUR)

    def to_c(self) -> N.ba_options:
        o = N.ba_options()
        o.max_num_iterations = int(self.max_num_iterations)
        o.max_num_consecutive_invalid_steps = int(self.max_num_consecutive_invalid_steps)
        o.jacobi_scaling = int(bool(self.jacobi_scaling))
        o.linear_solver = {"DENSE_SCHUR": 0, "ITERATIVE_SCHUR": 1}[self.linear_solver_type]
        o.preconditioner_type = {"JACOBI": 0, "SCHUR_JACOBI": 1}[self.preconditioner_type]
        o.max_linear_solver_iterations = int(self.max_linear_solver_iterations)
        o.min_linear_solver_iterations = int(self.min_linear_solver_iterations)
        o.precision = {"FP64": 0, "MIXED_FP32": 1}[self.precision]
        o.eta = float(self.eta)
        for f in ("function_tolerance", "gradient_tolerance", "parameter_tolerance",
                  "initial_trust_region_radius", "max_trust_region_radius", "min_trust_region_radius",
                  "min_relative_decrease", "min_lm_diagonal", "max_lm_diagonal"):
            setattr(o, f, float(getattr(self, f)))
        return o


@dataclass
class Summary:
    initial_cost: float
    final_cost: float
    num_iterations: int
    num_successful_steps: int
    num_unsuccessful_steps: int
    termination_type: str
    total_time_s: float
    linearize_time_s: float
    solve_time_s: float


ITER_FIELDS = [f for f, _ in N.ba_iteration._fields_]


class Solver:
    """A ba_ctx on one HIP device."""

    def __init__(self, device: int = 0):
        self.lib = N.load_library()
        h = C.c_void_p()
        st = self.lib.ba_create(C.byref(h), int(device))
        if st != N.BA_OK:
            raise N.BAError(st, f"ba_create(device={device}) failed")
        self.h = h
        self.problem: Problem | None = None
        self._keep = []

    def close(self):
        if getattr(self, "h", None):
            self.lib.ba_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st: int, what: str):
        if st != N.BA_OK:
            raise N.BAError(st, f"{what}: {self.lib.ba_last_error(self.h).decode(errors='replace')}")

    # -- multi-GPU ------------------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        lib = N.load_library()
        buf = C.create_string_buffer(128)
        st = lib.ba_comm_unique_id(buf)
        if st != N.BA_OK:
            raise N.BAError(st, "ba_comm_unique_id")
        return buf.raw

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        assert len(uid) == 128
        self._check(self.lib.ba_comm_init(self.h, C.c_char_p(uid), int(nranks), int(rank)), "ba_comm_init")

    def comm_init_host(self, allreduce, nranks: int, rank: int):
        """Host-staged transport for the multi-rank exchange (test hook, see
        ba_comm_init_host): `allreduce(values: np.ndarray, op: str)` reduces the
        float64 array in place across the ranks ("sum" / "max")."""
        def cb(_user, ptr, n, op):
            try:
                allreduce(np.ctypeslib.as_array(ptr, shape=(int(n),)), "max" if op == 1 else "sum")
                return 0
            except Exception:   # noqa: BLE001 - reported as BA_ERR_COMM
                return 1
        self._host_cb = N.HOST_ALLREDUCE_FN(cb)   # kept alive with the solver
        self._check(self.lib.ba_comm_init_host(self.h, C.cast(self._host_cb, C.c_void_p), None, int(nranks),
                                               int(rank)), "ba_comm_init_host")

    def allreduce_host(self, values, op: str = "sum") -> np.ndarray:
        """In-place RCCL reduction of a few host doubles across ranks (identity
        without a communicator)."""
        v = np.ascontiguousarray(values, dtype=np.float64).copy()
        self._check(self.lib.ba_comm_allreduce_host(self.h, _ptr(v), int(v.size), 0 if op == "sum" else 1),
                    "ba_comm_allreduce_host")
        return v

    def barrier(self):
        self._check(self.lib.ba_comm_allreduce_host(self.h, None, 0, 0), "ba_comm_allreduce_host")

    # -- problem ----------------------------------------------------------
    def set_problem(self, problem: Problem):
        p = problem.normalized()
        s = N.ba_problem()
        s.n_cams, s.n_pts, s.n_obs = p.n_cams, p.n_pts, p.n_obs
        s.cams, s.K, s.pts = _ptr(p.cams), _ptr(p.K), _ptr(p.pts)
        s.cam_fixed, s.cam_fixed_extr, s.pt_fixed = _ptr(p.cam_fixed), _ptr(p.cam_fixed_extr), _ptr(p.pt_fixed)
        s.obs_cam, s.obs_pt, s.obs_uv = _ptr(p.obs_cam), _ptr(p.obs_pt), _ptr(p.obs_uv)
        s.huber_a = p.huber_a
        self._check(self.lib.ba_set_problem(self.h, C.byref(s)), "ba_set_problem")
        self.problem = p

    def set_params(self, cams: np.ndarray | None, pts: np.ndarray | None):
        c = None if cams is None else np.ascontiguousarray(cams, np.float64)
        q = None if pts is None else np.ascontiguousarray(pts, np.float64)
        self._check(self.lib.ba_set_params(self.h, _ptr(c), _ptr(q)), "ba_set_params")

    def solve(self, options: Options | None = None) -> Summary:
        o = (options or Options()).to_c()
        s = N.ba_summary()
        self._check(self.lib.ba_solve(self.h, C.byref(o), C.byref(s)), "ba_solve")
        return Summary(s.initial_cost, s.final_cost, s.num_iterations, s.num_successful_steps,
                       s.num_unsuccessful_steps, N.TERMINATION_NAMES.get(s.termination_type, str(s.termination_type)),
                       s.total_time_s, s.linearize_time_s, s.solve_time_s)

    def params(self) -> tuple[np.ndarray, np.ndarray]:
        p = self.problem
        cams = np.empty((p.n_cams, 6))
        pts = np.empty((p.n_pts, 3))
        self._check(self.lib.ba_get_params(self.h, _ptr(cams), _ptr(pts)), "ba_get_params")
        return cams, pts

    def iteration_log(self) -> list[dict]:
        n = self.lib.ba_get_iteration_log(self.h, None, 0)
        arr = (N.ba_iteration * max(n, 1))()
        self.lib.ba_get_iteration_log(self.h, arr, n)
        return [{f: getattr(arr[i], f) for f in ITER_FIELDS} for i in range(n)]

    def residuals(self) -> tuple[np.ndarray, float]:
        r = np.empty((self.problem.n_obs, 2))
        cost = C.c_double()
        self._check(self.lib.ba_eval_residuals(self.h, _ptr(r), C.byref(cost)), "ba_eval_residuals")
        return r, cost.value

    def linearize(self) -> tuple[np.ndarray, np.ndarray, float]:
        n = self.problem.n_obs
        r = np.empty((n, 2))
        J = np.empty((n, 2, 9))
        cost = C.c_double()
        self._check(self.lib.ba_linearize(self.h, _ptr(r), _ptr(J), C.byref(cost)), "ba_linearize")
        return r, J, cost.value

    def debug_blocks(self, radius: float = 1e4, with_s: bool = True) -> dict:
        """The blocks of one DENSE_SCHUR step at the current parameters
        (iteration-0 Jacobi scaling, trust-region radius `radius`), as the
        solve's own kernels form them (ba_debug_blocks): Hpp [n_pts, 6], gp
        [n_pts, 3], Hcc [n_cams, 21] (lower, row-major), gc [n_cams, 6], and
        with_s: the reduced system S [n, n] (lower triangle) and rhs [n]."""
        p = self.problem
        Hpp, gp = np.empty((p.n_pts, 6)), np.empty((p.n_pts, 3))
        Hcc, gc = np.empty((p.n_cams, 21)), np.empty((p.n_cams, 6))
        n = C.c_int(0)
        if with_s:   # size of the variable-camera system: ask first (S, rhs NULL)
            self._check(self.lib.ba_debug_blocks(self.h, float(radius), None, None, None, None, None, None,
                                                 C.byref(n)), "ba_debug_blocks")
        S = np.empty((n.value, n.value)) if with_s else None
        rhs = np.empty(n.value) if with_s else None
        self._check(self.lib.ba_debug_blocks(self.h, float(radius), _ptr(Hpp), _ptr(gp), _ptr(Hcc), _ptr(gc),
                                             _ptr(S) if with_s else None, _ptr(rhs) if with_s else None,
                                             C.byref(n)), "ba_debug_blocks")
        return {"Hpp": Hpp, "gp": gp, "Hcc": Hcc, "gc": gc, "S": S, "rhs": rhs, "n": n.value}

    def prune(self, extr, cam_center, K, obs_cam, obs_X, obs_uv, obs_inv_sigma, obs_dist) -> np.ndarray:
        """pruneCorrespondences (Optimizer.cpp:6-79) on the device for a batch of
        (keyframe, keypoint) pairs; returns a uint8 ba_prune_result per pair."""
        arrs = [np.ascontiguousarray(a, dtype=np.float32) for a in (extr, cam_center, K)]
        oc = np.ascontiguousarray(obs_cam, dtype=np.int32)
        oarrs = [np.ascontiguousarray(a, dtype=np.float32) for a in (obs_X, obs_uv, obs_inv_sigma, obs_dist)]
        n_cams, n_obs = arrs[0].size // 16, oc.size
        pp = N.ba_prune_problem(n_cams=n_cams, n_obs=n_obs, extr=_ptr(arrs[0]), cam_center=_ptr(arrs[1]),
                                K=_ptr(arrs[2]), obs_cam=_ptr(oc), obs_X=_ptr(oarrs[0]), obs_uv=_ptr(oarrs[1]),
                                obs_inv_sigma=_ptr(oarrs[2]), obs_dist=_ptr(oarrs[3]))
        out = np.empty(n_obs, np.uint8)
        self._check(self.lib.ba_prune(self.h, C.byref(pp), _ptr(out)), "ba_prune")
        return out

    def solve_pose_batch(self, obs_offset, cams, K, pts, obs_uv, options: Options | None = None,
                         huber_a: float = HUBER_A) -> tuple[np.ndarray, list[Summary]]:
        """Batched pose-only solves (MotionOnlyBAOptimizerAngles' Ceres solve,
        Optimizer.cpp:417-442, for many frames in one launch).  Problem i owns
        observations [obs_offset[i], obs_offset[i+1]) of constant points
        pts[o] with pixels obs_uv[o]; returns (cams (n, 6), summaries)."""
        off = np.ascontiguousarray(obs_offset, dtype=np.int32)
        n = off.size - 1
        c = np.ascontiguousarray(cams, dtype=np.float64).reshape(n, 6)
        k = np.ascontiguousarray(K, dtype=np.float32).reshape(n, 9)
        x = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 3)
        uv = np.ascontiguousarray(obs_uv, dtype=np.float32).reshape(-1, 2)
        b = N.ba_pose_batch(n_problems=n, reserved=0, obs_offset=_ptr(off), cams=_ptr(c), K=_ptr(k), pts=_ptr(x),
                            obs_uv=_ptr(uv), huber_a=float(huber_a))
        o = (options or Options()).to_c()
        out = np.empty((n, 6))
        sums = (N.ba_summary * max(n, 1))()
        self._check(self.lib.ba_solve_pose_batch(self.h, C.byref(b), C.byref(o), _ptr(out), sums),
                    "ba_solve_pose_batch")
        res = [Summary(s.initial_cost, s.final_cost, s.num_iterations, s.num_successful_steps,
                       s.num_unsuccessful_steps, N.TERMINATION_NAMES.get(s.termination_type, str(s.termination_type)),
                       s.total_time_s, s.linearize_time_s, s.solve_time_s) for s in list(sums)[:n]]
        return out, res

    def synchronize(self):
        self._check(self.lib.ba_synchronize(self.h), "ba_synchronize")

    def bench_iterations(self, iters: int, radius: float = 1e4, options: Options | None = None,
                         with_linear_iters: bool = False, time_rj: bool = True):
        """Device time of `iters` LM iterations at a fixed radius: returns
        (ms per iteration, ms of the residual+Jacobian kernel[, mean linear
        solver iterations per LM iteration]).  time_rj=False: no event pair
        around the residual+Jacobian kernel (its ms is then None)."""
        ms = C.c_double()
        rj = C.c_double()
        li = C.c_double()
        o = (options or Options()).to_c()
        self._check(self.lib.ba_bench_iterations(self.h, C.byref(o), int(iters), float(radius), C.byref(ms),
                                                 C.byref(rj) if time_rj else None, C.byref(li)),
                    "ba_bench_iterations")
        r = rj.value if time_rj else None
        if with_linear_iters:
            return ms.value, r, li.value
        return ms.value, r

    def bench_iteration_times(self) -> np.ndarray:
        """Host wall time (ms) of each LM iteration of the last
        bench_iterations call (scalar record to scalar record)."""
        n = self.lib.ba_bench_iteration_times(self.h, None, 0)
        out = np.empty(max(n, 0))
        if n > 0:
            self.lib.ba_bench_iteration_times(self.h, _ptr(out), n)
        return out

    def stream_copy(self, nbytes: int = 1 << 30, reps: int = 10) -> float:
        """Measured device copy bandwidth in GB/s (read + write bytes), the
        STREAM-copy figure SURVEY.md §8d asks for beside the HBM peak."""
        g = C.c_double()
        self._check(self.lib.ba_stream_copy(self.h, C.c_size_t(int(nbytes)), int(reps), C.byref(g)), "ba_stream_copy")
        return g.value


def solve(problem: Problem, options: Options | None = None, device: int = 0):
    """One-shot convenience: returns (cams, pts, summary, iteration_log)."""
    with Solver(device) as s:
        s.set_problem(problem)
        summ = s.solve(options)
        cams, pts = s.params()
        return cams, pts, summ, s.iteration_log()
