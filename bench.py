#!/usr/bin/env python3
"""bench.py — M-obs/s per LM iteration (residual+Jacobian+Schur) on MI355X.

One "step" = one full Levenberg-Marquardt iteration of the reference's Ceres
DENSE_SCHUR path (ba_project/src/ba/Optimizer.cpp:80-90): linearise (r, J,
Huber), assemble the block normal equations, eliminate the points, form and
factor the reduced camera system, back-substitute, evaluate the model cost
change and the candidate cost — the accept/reject scalars read back to the
host exactly as the solver does.  Inputs are resident in HBM before timing.

Workload (N=1): BASELINE.json configs[2] = synthetic BAL-style 200 cams x
100k points x 1M observations ("C3", the single-GPU config the metric is
quoted on).  N>1: weak scaling — every rank owns a disjoint 100k-point shard
(1M observations) of one scene with the same 200 replicated cameras; the
camera-side system is all-reduced over RCCL each iteration.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1 via python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(config: str):
    """Per-launch HBM bytes of the residual+Jacobian kernel from the committed
    rocprofv3 PMC summary (profiles/), corrected per MI355X_MICROARCH.md
    (FETCH_SIZE x2 on gfx950), or None."""
    f = ROOT / "profiles" / f"pmc_{config}.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        return float(d["k_linearize"]["hbm_bytes_per_launch"])
    except Exception:
        return None


def uid_path(world: int) -> Path:
    """Rendezvous file of one launch: keyed by the launcher (torch.distributed.run
    is the parent of every rank) and its master port."""
    key = f"{os.environ.get('MASTER_ADDR', '127.0.0.1')}_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}_{world}"
    return Path(tempfile.gettempdir()) / f"ba_rccl_uid_{key}.bin"


def rendezvous_uid(rank: int, world: int, timeout_s: float = 300.0) -> bytes:
    from bundleadjustment_amd import Solver
    path = uid_path(world)
    if rank == 0:
        uid = Solver.unique_id()
        tmp = path.with_name(path.name + f".{os.getpid()}.tmp")
        tmp.write_bytes(uid)
        os.replace(tmp, path)          # atomic publish
        return uid
    deadline = time.time() + timeout_s
    while time.time() < deadline:
        try:
            data = path.read_bytes()
            if len(data) == 128:
                return data
        except FileNotFoundError:
            pass
        time.sleep(0.05)
    raise RuntimeError(f"rank {rank}: no RCCL id at {path} after {timeout_s:.0f} s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--scale", type=float, default=1.0, help="point-count scale of the config (per-GPU shard size)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    ap.add_argument("--comm", action="store_true", help="use an RCCL communicator even at one rank (tests)")
    ap.add_argument("--linear-solver", default="dense", choices=["dense", "iterative"],
                    help="DENSE_SCHUR (the reference's) or ITERATIVE_SCHUR (implicit Schur + PCG)")
    ap.add_argument("--preconditioner", default="SCHUR_JACOBI", choices=["JACOBI", "SCHUR_JACOBI"])
    ap.add_argument("--precision", default="FP64", choices=["FP64", "MIXED_FP32"],
                    help="MIXED_FP32: fp32 storage of the per-observation Schur blocks (iterative only)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    import numpy as np

    from bundleadjustment_amd import Options, Solver, make_config
    from bundleadjustment_amd.problem import CONFIG_INDEX, CONFIGS

    cfg = args.config
    seed = 0xBA5E0000 + CONFIG_INDEX[cfg]
    t = time.time()
    problem = make_config(cfg, scale=args.scale, point_seed=None if rank == 0 else seed + 7919 * rank)
    log(f"[rank {rank}] problem {cfg}: {problem.n_cams} cams x {problem.n_pts} pts x {problem.n_obs} obs "
        f"(generated in {time.time() - t:.1f}s)")

    solver = Solver(local_rank)
    use_comm = world > 1 or args.comm
    if use_comm:
        # RCCL communicator; the 128-byte id travels through a file keyed by the
        # launcher (no second GPU runtime in this process for the rendezvous)
        uid = rendezvous_uid(rank, world)
        solver.comm_init(uid, world, rank)
        if rank == 0:
            uid_path(world).unlink(missing_ok=True)
    solver.set_problem(problem)

    def barrier():
        if use_comm:
            solver.barrier()

    iterative = args.linear_solver == "iterative"
    opts = Options(linear_solver_type="ITERATIVE_SCHUR" if iterative else "DENSE_SCHUR",
                   preconditioner_type=args.preconditioner, precision=args.precision)
    # warmup (first call also computes the Jacobi scaling, as LM iteration 0 does)
    solver.bench_iterations(max(1, args.warmup), options=opts)
    barrier()
    solver.synchronize()
    t0 = time.perf_counter()
    ms_dev, ms_rj, cg_iters = solver.bench_iterations(args.steps, options=opts, with_linear_iters=True)
    solver.synchronize()
    barrier()
    dt = time.perf_counter() - t0

    n_obs_total = problem.n_obs
    if use_comm:   # max over ranks of the timed region, total observations
        dt = float(solver.allreduce_host([dt], "max")[0])
        n_obs_total = int(solver.allreduce_host([float(problem.n_obs)], "sum")[0])

    # algorithmic bytes of the residual+Jacobian kernel per launch:
    #   176 B/obs (uv 8 + two int32 idx 8 + r 16 + J 144) + 24 B/point + 48 B/camera
    B_rj = 176.0 * problem.n_obs + 24.0 * problem.n_pts + 48.0 * problem.n_cams
    achieved = B_rj / (ms_rj * 1e-3) / 1e9
    traffic = pmc_traffic(cfg)
    roofline = {"kernel": "k_linearize (residual+Jacobian)", "bound": "hbm", "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "algorithmic_bytes": B_rj, "avg_launch_ms": round(ms_rj, 5)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle
        oracle.build()
        threads = min(16, os.cpu_count() or 1)
        oracle.set_threads(threads)
        first = oracle.bench_seconds_per_iteration(problem, 1)
        iters = max(1, min(30, int(args.cpu_seconds / max(first, 1e-3))))
        spi = oracle.bench_seconds_per_iteration(problem, iters)
        cpu = {"value": round(problem.n_obs / spi / 1e6, 3), "unit": "M-obs/s", "cores": threads, "kind": "port",
               "sample": f"full {cfg} problem ({problem.n_obs} obs), {iters} LM iterations of the C++ CPU "
                         f"restatement of Ceres LM+DENSE_SCHUR (oracle/), not Ceres; {spi:.3f} s/iteration"}

    if rank == 0:
        ms_step = dt / args.steps * 1e3
        out = {
            "metric": "M-obs/s per LM iteration (residual+Jacobian+Schur)",
            "value": round(n_obs_total * args.steps / dt / 1e6, 2),
            "unit": "M-obs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (BAL-style, SURVEY.md §8d generator, seeded)",
            "config": {"workload": f"{cfg.upper()}: {CONFIGS[cfg]['n_cams']} cams x {problem.n_pts} pts x "
                                   f"{problem.n_obs} obs per GPU (point-sharded, cameras replicated)",
                       "global_obs": n_obs_total,
                       "solver": (f"LM + ITERATIVE_SCHUR (implicit Schur, PCG {args.preconditioner}, "
                                  f"{cg_iters:.1f} CG iterations per LM iteration), fp64"
                                  + (", W blocks stored fp32" if args.precision == "MIXED_FP32" else "")) if iterative
                       else "LM + DENSE_SCHUR, fp64",
                       "parallelism": f"points sharded x{world}, RCCL all-reduce of "
                                      + ("camera blocks + one 6C vector per CG iteration" if iterative
                                         else "camera system")},
            "device_ms_per_step": round(ms_dev, 4),
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    solver.close()


if __name__ == "__main__":
    main()
