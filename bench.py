#!/usr/bin/env python3
"""bench.py — M-obs/s per LM iteration (residual+Jacobian+Schur) on MI355X.

One "step" = one full Levenberg-Marquardt iteration of the reference's Ceres
DENSE_SCHUR path (ba_project/src/ba/Optimizer.cpp:80-90): linearise (r, J,
Huber), assemble the block normal equations, eliminate the points, form and
factor the reduced camera system, back-substitute, evaluate the model cost
change and the candidate cost — the accept/reject scalars read back to the
host exactly as the solver does.  Inputs are resident in HBM before timing.

Workloads (--workload):
  c3   (default) BASELINE.json configs[2], synthetic BAL-style 200 cams x 100k
       points x 1M observations per GPU, DENSE_SCHUR (the reference's solver).
       N = 1 is the single-GPU roofline config the metric is quoted on; N > 1
       is weak scaling: every rank owns a disjoint 100k-point shard of one
       scene with the same 200 replicated cameras, the camera-side system is
       all-reduced over RCCL each iteration.
  c4   BASELINE.json configs[3]: ONE fixed 1k cams x 1M points x 10M
       observations problem split over the N ranks (strong scaling; the
       points come in 8 fixed blocks of 125k, rank r holds blocks r, r + N,
       ...), ITERATIVE_SCHUR (implicit Schur, no 6000^2 system per rank; one
       6C all-reduce per CG iteration).
  c5   BASELINE.json configs[4]: 10k cams x 10M points x 100M observations
       (8 blocks of 1.25M points), ITERATIVE_SCHUR with the W blocks stored in
       fp32 (BA_MIXED_FP32).

Default workload: c3 at N = 1 (the single-GPU roofline config), c4 at N > 1
(BASELINE configs[3], the multi-GPU config).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c4|c5]
  N > 1 either under a launcher (python -m torch.distributed.run
  --nproc-per-node N bench.py --gpus N ...: RANK / LOCAL_RANK / WORLD_SIZE set,
  WORLD_SIZE must equal N) or standalone: without WORLD_SIZE the process
  starts N rank processes itself (before touching the GPU), rank r on device
  r, and relays rank 0's JSON line.
  --transport host: the exchange goes through torch.distributed gloo on the
  host instead of RCCL (several ranks on one GPU, tests; --device pins every
  rank to one device).
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


def pmc_record(config: str, kernel: str, n_obs: int, scale: float = 1.0):
    """Per-launch HBM bytes (and VALU instructions, when recorded) of the
    residual+Jacobian kernel from a committed rocprofv3 PMC summary
    (profiles/pmc_<config>*.json, tools/pmc_summary.py: separate FETCH_SIZE /
    WRITE_SIZE passes, FETCH_SIZE x2 per MI355X_MICROARCH.md's gfx950
    correction).  A summary measured on a problem of another size (its
    "_problem" n_obs) is scaled linearly in the observations and says so; a
    summary without a recorded size counts only for the full-size c3 run it
    was taken on.  None when no summary covers the kernel."""
    best = None
    for f in sorted((ROOT / "profiles").glob(f"pmc_{config}*.json")):
        try:
            d = json.loads(f.read_text())
            k = d[kernel]
            n_at = (d.get("_problem") or {}).get("n_obs")
            if n_at is None and not (config == "c3" and scale == 1.0 and f.name == "pmc_c3.json"):
                continue
            n_at = n_at or n_obs
            cand = (abs(n_at - n_obs), f.name, k, n_at)
        except Exception:
            continue
        if best is None or cand[0] < best[0]:
            best = cand
    if best is None:
        return None
    _, name, k, n_at = best
    f = n_obs / n_at
    rec = {"hbm_bytes_per_launch": float(k["hbm_bytes_per_launch"]) * f,
           "source": f"profiles/{name}" + ("" if n_at == n_obs else f" (measured at {n_at} obs, scaled x{f:.4g})")}
    if k.get("valu_insts_per_launch"):
        rec["valu_insts_per_launch"] = float(k["valu_insts_per_launch"]) * f
    return rec


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


STRONG = {   # global problems of the strong-scaling workloads: 8 fixed point blocks
    "c4": dict(blocks=8, solver="ITERATIVE_SCHUR", precision="FP64"),
    "c5": dict(blocks=8, solver="ITERATIVE_SCHUR", precision="MIXED_FP32"),
}


def strong_shard(cfg: str, rank: int, world: int, scale: float = 1.0):
    """Rank `rank`'s part of the fixed global problem of `cfg`: point blocks
    b = rank, rank + world, ... of 8 (block b drawn with point_seed
    seed + 7919 b over the shared cameras), concatenated.  The union over the
    ranks is the same problem for every N that divides 8."""
    import numpy as np
    from bundleadjustment_amd import make_config
    from bundleadjustment_amd.problem import CONFIG_INDEX
    nb = STRONG[cfg]["blocks"]
    seed = 0xBA5E0000 + CONFIG_INDEX[cfg]
    parts = [make_config(cfg, scale=scale / nb, point_seed=seed + 7919 * b) for b in range(rank, nb, world)]
    p = parts[0].copy()
    off = np.cumsum([0] + [q.n_pts for q in parts])
    p.pts = np.concatenate([q.pts for q in parts])
    p.obs_cam = np.concatenate([q.obs_cam for q in parts])
    p.obs_pt = np.concatenate([q.obs_pt + o for q, o in zip(parts, off)]).astype(np.int32)
    p.obs_uv = np.concatenate([q.obs_uv for q in parts])
    p.gt_pts = None
    return p.normalized()


def cpu_baseline_leg(problem, cfg: str, target_s: float, precision: str = "FP64"):
    """The oracle (C++ restatement of Ceres LM, not Ceres) on the host cores:
    at the reference's num_threads = 4 (Optimizer.cpp:88) and at every thread
    this process may use (OMP_NUM_THREADS, else os.cpu_count()).  DENSE_SCHUR
    (the reference's solver) up to 2000 cameras; beyond, where a dense 6C x 6C
    system is infeasible (C5: 60000^2), its ITERATIVE_SCHUR restatement, timed
    as one-iteration solves (initial linearisation + one LM step)."""
    import oracle
    oracle.build()
    nproc = os.cpu_count() or 1
    allowed = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or nproc
    iterative = problem.n_cams > 2000

    def leg(threads):
        oracle.set_threads(threads)
        if iterative:
            o = oracle.default_options(max_num_iterations=1, linear_solver=1, preconditioner_type=1,
                                       precision=1 if precision == "MIXED_FP32" else 0)
            t0 = time.perf_counter()
            oracle.solve(problem, o)
            return time.perf_counter() - t0, 1
        first = oracle.bench_seconds_per_iteration(problem, 1)
        iters = max(1, min(30, int(target_s / max(first, 1e-3))))
        return oracle.bench_seconds_per_iteration(problem, iters), iters

    spi4, it4 = leg(min(4, allowed))
    spia, ita = leg(allowed) if allowed != min(4, allowed) else (spi4, it4)
    solver = ("ITERATIVE_SCHUR (SCHUR_JACOBI" + (", fp32 W" if precision == "MIXED_FP32" else "") +
              "; one-iteration solves: initial linearisation + one LM step)") if iterative else "DENSE_SCHUR"
    return {"value": round(problem.n_obs / spia / 1e6, 3), "unit": "M-obs/s", "cores": allowed, "kind": "port",
            "sample": f"full {cfg} problem ({problem.n_obs} obs), {ita} LM iteration(s) of the C++ CPU restatement "
                      f"of Ceres LM + {solver} (oracle/), not Ceres; {spia:.3f} s/iteration at {allowed} threads "
                      f"(host nproc {nproc})",
            "nproc": nproc,
            "reference_threads": {"threads": min(4, allowed), "value": round(problem.n_obs / spi4 / 1e6, 3),
                                  "s_per_iteration": round(spi4, 4), "iterations": it4,
                                  "note": "num_threads = 4 as configureSolver sets it (Optimizer.cpp:88)"}}


def free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n: int, argv: list[str], timeout_s: float | None = None) -> int:
    """Standalone N > 1: start N copies of this script as ranks 0..N-1 (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT set), rank 0's
    stdout relayed as ours, every rank's stderr passed through.  Runs before
    anything in this process touches the GPU (the ranks own the devices).
    Returns the first non-zero exit status (the other ranks are then
    terminated), else 0."""
    import subprocess
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + argv, env=env,
                                      stdout=None if r == 0 else sys.stderr))
    deadline = None if timeout_s is None else time.time() + timeout_s
    rc = 0
    pending = list(procs)
    while pending:
        for pr in list(pending):
            code = pr.poll()
            if code is None:
                continue
            pending.remove(pr)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:   # a failed rank would leave the others waiting in a collective
                    q.terminate()
        if deadline is not None and time.time() > deadline:
            for q in pending:
                q.kill()
            rc = rc or 124
            break
        time.sleep(0.05)
    for pr in procs:
        pr.wait()
    return rc


def host_transport(rank: int, world: int):
    """gloo process group for --transport host (the ba_comm_init_host hook)."""
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allreduce(v, op):
        dist.all_reduce(torch.from_numpy(v), op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return allreduce


def dry_run_line(args, rank, world, local_rank, device):
    """BA_BENCH_DRYRUN=1 (CPU tests of the launch logic): what this rank would
    run, without any GPU call."""
    return json.dumps({"dry_run": True, "rank": rank, "world": world, "local_rank": local_rank, "device": device,
                       "workload": args.workload, "transport": args.transport, "steps": args.steps,
                       "warmup": args.warmup, "mode": args.mode})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default=None, choices=["c3", "c4", "c5"],
                    help="c3: weak scaling of configs[2] (default at N = 1); c4 / c5: strong scaling of "
                         "configs[3] / [4] (c4 is the default at N > 1)")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "host"],
                    help="multi-rank exchange: RCCL over xGMI (default) or host-staged through gloo (tests)")
    ap.add_argument("--device", type=int, default=None, help="HIP device of every rank (default: LOCAL_RANK)")
    ap.add_argument("--config", default=None, help="weak mode: per-GPU config (default c3)")
    ap.add_argument("--scale", type=float, default=1.0,
                    help="point-count scale of the problem (weak: of the per-GPU shard; strong: of the global "
                         "problem); 1 = the BASELINE size")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target length of each CPU-baseline sample")
    ap.add_argument("--comm", action="store_true", help="use an RCCL communicator even at one rank (tests)")
    ap.add_argument("--linear-solver", default=None, choices=["dense", "iterative"],
                    help="DENSE_SCHUR (the reference's) or ITERATIVE_SCHUR (implicit Schur + PCG)")
    ap.add_argument("--preconditioner", default="SCHUR_JACOBI", choices=["JACOBI", "SCHUR_JACOBI"])
    ap.add_argument("--precision", default=None, choices=["FP64", "MIXED_FP32"],
                    help="MIXED_FP32: fp32 storage of the per-observation Schur blocks (iterative only)")
    ap.add_argument("--mode", default=None, choices=["fixed", "trajectory"],
                    help="fixed: every step re-linearises at x0 and takes a trial step at the initial radius "
                         "(identical work per step; default for c3, whose DENSE_SCHUR step does not depend on the "
                         "radius); trajectory: ONE ba_solve from x0 for exactly K LM iterations with Ceres' radius "
                         "schedule (accepted and rejected steps, the CG counts the radius implies; default for "
                         "c4 / c5)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {args.gpus})")
    if args.workload is None:
        args.workload = "c3" if args.gpus == 1 else "c4"
    if args.mode is None:
        args.mode = "trajectory" if args.workload in STRONG else "fixed"

    if args.workload in STRONG and 8 % args.gpus != 0:
        raise SystemExit(f"--workload {args.workload}: the 8 point blocks need a rank count dividing 8 "
                         f"(got {args.gpus})")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:   # standalone N > 1: this process only launches and relays
            sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
        world, rank, local_rank = 1, 0, 0
    else:
        world = int(os.environ["WORLD_SIZE"])
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
        if world != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a {world}-rank run "
                             f"as {args.gpus} GPU(s)")
    device = local_rank if args.device is None else args.device
    # the JSON line is the only thing a rank writes to stdout: native
    # libraries print there too (RCCL's version banner at communicator
    # creation), so fd 1 goes to stderr and the line to a copy of the original
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if os.environ.get("BA_BENCH_DRYRUN") == "1":
        if os.environ.get("BA_BENCH_DRYRUN_FAIL_RANK") == str(rank):
            raise SystemExit(3)
        print(dry_run_line(args, rank, world, local_rank, device), file=json_out, flush=True)
        if rank != 0:   # a surviving rank of a failed launch is terminated by the parent
            time.sleep(float(os.environ.get("BA_BENCH_DRYRUN_SLEEP", "0")))
        return

    import numpy as np

    from bundleadjustment_amd import Options, Solver, make_config
    from bundleadjustment_amd.problem import CONFIG_INDEX, CONFIGS

    strong = args.workload in STRONG
    cfg = args.workload if strong else (args.config or "c3")
    seed = 0xBA5E0000 + CONFIG_INDEX[cfg]
    t = time.time()
    if strong:
        problem = strong_shard(cfg, rank, world, args.scale)
    else:
        problem = make_config(cfg, scale=args.scale, point_seed=None if rank == 0 else seed + 7919 * rank)
    log(f"[rank {rank}] problem {cfg}: {problem.n_cams} cams x {problem.n_pts} pts x {problem.n_obs} obs "
        f"(generated in {time.time() - t:.1f}s)")

    use_comm = world > 1 or args.comm
    # host transport: the gloo group comes up before this process's first HIP
    # call and is torn down after the solver (as tests/mr_worker.py does)
    host_ar = host_transport(rank, world) if use_comm and args.transport == "host" else None
    solver = Solver(device)
    if host_ar is not None:
        solver.comm_init_host(host_ar, world, rank)
    elif use_comm:
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

    lin = args.linear_solver or ("iterative" if strong else "dense")
    precision = args.precision or (STRONG[cfg]["precision"] if strong else "FP64")
    iterative = lin == "iterative"
    opts = Options(linear_solver_type="ITERATIVE_SCHUR" if iterative else "DENSE_SCHUR",
                   preconditioner_type=args.preconditioner, precision=precision)
    trajectory = None
    rj_in_loop = os.environ.get("BENCH_RJ_IN_LOOP") == "1"
    if args.mode == "trajectory":
        # ONE solve from x0 for exactly K LM iterations: Ceres' radius
        # schedule (x3 per good step, /2, /4 ... per rejected one), so each
        # step's CG count is the one its radius implies (2-7 on this
        # generator) and rejected steps skip the re-linearisation.  The
        # termination tests are off so that K iterations run; nothing else
        # differs from ba_solve with configureSolver's options.
        import dataclasses
        x0c, x0p = solver.problem.cams.copy(), solver.problem.pts.copy()
        topts = dataclasses.replace(opts, max_num_iterations=args.steps, function_tolerance=0.0,
                                    gradient_tolerance=0.0, parameter_tolerance=0.0)
        # warmup: a W-iteration solve (buffers, Jacobi scaling), then back to x0
        solver.solve(dataclasses.replace(topts, max_num_iterations=max(1, args.warmup)))
        solver.set_params(x0c, x0p)
        barrier()
        solver.synchronize()
        t0 = time.perf_counter()
        summ = solver.solve(topts)
        solver.synchronize()
        barrier()
        dt = time.perf_counter() - t0
        tlog = solver.iteration_log()[1:]          # [0] is the initial linearisation
        it_ms = np.array([r["iteration_time_s"] * 1e3 for r in tlog])
        cg = [int(r["linear_solver_iterations"]) for r in tlog]
        cg_iters = float(np.mean(cg)) if cg else 0.0
        # where Ceres' default function tolerance (1e-6 relative cost change)
        # would have ended the solve
        stop = next((i + 1 for i, r in enumerate(tlog) if r["step_is_successful"]
                     and abs(r["cost_change"]) <= 1e-6 * (r["cost"] + r["cost_change"])), None)
        productive = float(np.mean(it_ms[:stop])) if stop else None
        trajectory = {"lm_iterations": summ.num_iterations, "successful_steps": summ.num_successful_steps,
                      "unsuccessful_steps": summ.num_unsuccessful_steps,
                      "initial_cost": summ.initial_cost, "final_cost": summ.final_cost,
                      "linear_solver_iterations": cg,
                      "iteration_ms": [round(float(x), 4) for x in it_ms],
                      "ceres_default_function_tolerance_stop": stop,
                      "ms_per_iteration_to_that_stop": round(productive, 4) if productive else None,
                      "linear_solver_iterations_to_that_stop": (round(float(np.mean(cg[:stop])), 2) if stop
                                                                 else None),
                      "note": "one ba_solve from x0 (termination tests off, Ceres' radius schedule); ms_per_step "
                              "= the solve's wall time / its LM iterations, initial linearisation included"}
        steps_done = summ.num_iterations
        ms_dev = dt / max(steps_done, 1) * 1e3
        # the r+J kernel's launch time does not depend on the radius: timed in
        # a short fixed-radius pass after the solve
        _, ms_rj = solver.bench_iterations(min(args.steps, 10), options=opts)
        barrier()
    else:
        # warmup (first call also computes the Jacobi scaling, as LM iteration 0 does)
        solver.bench_iterations(max(1, args.warmup), options=opts)
        barrier()
        solver.synchronize()
        # the timed region carries no event pair around the r+J kernel (each
        # pair's packets idle the device ~5 us per LM iteration); the kernel is
        # timed with HIP events on its stream in a second pass of the same K
        # iterations right after (BENCH_RJ_IN_LOOP=1: both in one pass, A/B)
        t0 = time.perf_counter()
        ms_dev, ms_rj, cg_iters = solver.bench_iterations(args.steps, options=opts, with_linear_iters=True,
                                                          time_rj=rj_in_loop)
        solver.synchronize()
        barrier()
        dt = time.perf_counter() - t0
        steps_done = args.steps
        # per-iteration host wall times of the timed region (the
        # median of >= 10 iterations after 2 warm-ups), reported beside the mean
        it_ms = solver.bench_iteration_times()
        if not rj_in_loop:
            _, ms_rj = solver.bench_iterations(args.steps, options=opts)
            barrier()

    n_obs_total = problem.n_obs
    n_pts_total = problem.n_pts
    if use_comm:   # max over ranks of the timed region, total observations
        dt = float(solver.allreduce_host([dt], "max")[0])
        if len(it_ms):   # the slowest rank per iteration
            it_ms = np.asarray(solver.allreduce_host(list(it_ms), "max"))
        tot = solver.allreduce_host([float(problem.n_obs), float(problem.n_pts)], "sum")
        n_obs_total, n_pts_total = int(tot[0]), int(tot[1])

    # algorithmic bytes of the residual+Jacobian kernel per launch:
    #   176 B/obs (uv 8 + two int32 idx 8 + r 16 + J 144) + 24 B/point + 48 B/camera
    # and, with fp32 storage (MIXED_FP32, the C5 configuration), §8d's
    #   96 B/obs (r 8 + J 72 + uv 8 + idx 8) + 12 B/point + 24 B/camera
    mixed = precision == "MIXED_FP32"
    N, Pn, Cn = float(problem.n_obs), float(problem.n_pts), float(problem.n_cams)
    B_rj = (96.0 * N + 12.0 * Pn + 24.0 * Cn) if mixed else (176.0 * N + 24.0 * Pn + 48.0 * Cn)
    achieved = B_rj / (ms_rj * 1e-3) / 1e9
    # J-free iteration (libba_hip's default, BA_JR unset): the timed kernel is
    # k_lin_point, which forms r and J in registers and reduces them into the
    # point blocks without storing J (camera table in LDS up to 200 cameras,
    # the L2-resident global table beyond); SURVEY.md §8d prices such a fused
    # kernel against the unfused B_rj, labelled "effective"
    jrfree = os.environ.get("BA_JR") != "1"
    kname = ("k_lin_point" if problem.n_cams <= 200 else "k_lin_point_d") if jrfree else "k_linearize"
    pmc = pmc_record(cfg, kname, problem.n_obs, args.scale)
    traffic = pmc["hbm_bytes_per_launch"] if pmc else None
    # measured copy bandwidth of this GPU (reported beside the
    # vendor peak, which stays the denominator of `frac`): 1 GiB non-temporal
    # 16-B copy, 10 launches, after the timed region
    copy_gbs = solver.stream_copy(1 << 30, 10)
    roofline = {"kernel": (f"{kname} (residual + Jacobian + Huber + point blocks; J not materialised)" if jrfree
                           else "k_linearize (residual+Jacobian)"),
                "effective": jrfree,
                "bound": "hbm", "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "algorithmic_bytes": B_rj,
                "algorithmic_formula": ("96 N + 12 P + 24 C (fp32 r + J storage, SURVEY.md §8d)" if mixed
                                        else "176 N + 24 P + 48 C (fp64 r + J, SURVEY.md §8d)"),
                "avg_launch_ms": round(ms_rj, 5),
                "timing": ("HIP events around every launch, in the timed region" if rj_in_loop else
                           "HIP events around every launch, in a second pass of the same K LM iterations"
                           if args.mode == "fixed" else
                           "HIP events around every launch, in a fixed-radius pass after the trajectory"),
                "measured_copy": round(copy_gbs, 1), "frac_of_copy": round(achieved / copy_gbs, 4)}
    if jrfree:
        roofline["effective_note"] = (
            "J is never stored: the kernel moves far fewer bytes than the unfused B_rj it is priced against, so "
            "'achieved' and 'frac_of_copy' (> 1 possible) are bookkeeping, not a bandwidth claim; the kernel's "
            "real HBM rate is 'real'")
    if pmc:
        real = pmc["hbm_bytes_per_launch"] / (ms_rj * 1e-3) / 1e9
        roofline["real"] = {"hbm_bytes_per_launch": pmc["hbm_bytes_per_launch"], "achieved": round(real, 1),
                            "frac": round(real / HBM_PEAK_GBS, 4), "source": pmc["source"]}
        if pmc.get("valu_insts_per_launch"):
            # fp64 VALU issue: a wave64 fp64 instruction holds its SIMD's 16
            # fp64 lanes 4 cycles; 4 SIMDs x 256 CUs at the 2.4 GHz peak clock
            # (4 cycles per wave64 VALU instruction on a 16-lane SIMD)
            busy = pmc["valu_insts_per_launch"] * 4.0 / (ms_rj * 1e-3 * 2.4e9 * 1024.0)
            roofline["real"]["valu_insts_per_launch"] = pmc["valu_insts_per_launch"]
            roofline["real"]["valu_busy_frac_est"] = round(busy, 4)

    # whole-iteration figure (reported beside the kernel line):
    # B_iter = 176N (r+J) + 160N (r, J re-read for assembly) + 144N (W write)
    # + 144N (W read, Schur) + 16N (candidate: uv + idx) + P (24 + 72 + 72)
    # + C (48 + 216) + 16 (6C)^2 (dense S formed and factored) or 2 x 144N per
    # CG iteration (implicit Schur); W terms 72N with fp32 W storage.  Per
    # rank, over the rank's device time per LM iteration.
    wb = 72.0 if mixed else 144.0
    B_iter = (176.0 + 160.0 + 2.0 * wb + 16.0) * N + 168.0 * Pn + 264.0 * Cn
    B_iter += 2.0 * wb * N * cg_iters if iterative else 16.0 * (6.0 * Cn) ** 2
    it_ach = B_iter / (ms_dev * 1e-3) / 1e9
    iteration_roofline = {"bound": "hbm", "achieved": round(it_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(it_ach / HBM_PEAK_GBS, 4), "algorithmic_bytes": round(B_iter),
                          "note": "B_iter of SURVEY.md §8d over the device time per LM iteration (one rank); " +
                                  ("the implicit-Schur iteration runs a chain of streaming kernels (W, "
                                   "matvecs, camera-order gathers through the Infinity Cache) at 0.3-0.6 of "
                                   "HBM each" if iterative else
                                   "the iteration is bound by the serial reduced-camera factorisation and the "
                                   "Infinity-Cache Schur gathers, not by HBM")}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if problem.n_obs <= 20_000_000:
            cpu = cpu_baseline_leg(problem, cfg, args.cpu_seconds, precision)
        else:   # one CPU LM iteration alone would take minutes: no bounded sample
            log(f"cpu baseline skipped: {problem.n_obs} observations")

    if rank == 0:
        ms_step = dt / steps_done * 1e3
        mixed = precision == "MIXED_FP32"
        if strong:
            workload = (f"{cfg.upper()}: one {CONFIGS[cfg]['n_cams']} cams x {n_pts_total} pts x {n_obs_total} obs "
                        f"problem split over {world} GPU(s) (8 fixed point blocks, cameras replicated)")
        else:
            workload = (f"{cfg.upper()}: {CONFIGS[cfg]['n_cams']} cams x {problem.n_pts} pts x {problem.n_obs} obs "
                        f"per GPU (point-sharded, cameras replicated)")
        if iterative:
            exchange = "one folded 6C-double vector per CG iteration + the camera blocks per LM iteration"
            solver_s = (f"LM + ITERATIVE_SCHUR (implicit Schur, PCG {args.preconditioner}, {cg_iters:.1f} CG "
                        f"iterations per LM iteration), fp64" + (", W blocks stored fp32" if mixed else ""))
        else:
            exchange = "the packed reduced camera system (n(n+1)/2 + n doubles) + the camera blocks per LM iteration"
            solver_s = "LM + DENSE_SCHUR, fp64"
        out = {
            "metric": "M-obs/s per LM iteration (residual+Jacobian+Schur)",
            "value": round(n_obs_total * steps_done / dt / 1e6, 2),
            "unit": "M-obs/s",
            "n_gpus": world,
            "steps": steps_done,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "ms_per_step_median": round(float(np.median(it_ms)), 4) if len(it_ms) else None,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64 (W blocks f32)" if mixed else "f64",
            "data": "synthetic (BAL-style, SURVEY.md §8d generator, seeded)",
            "config": {"workload": workload,
                       "global_obs": n_obs_total,
                       "scale": args.scale,
                       "solver": solver_s,
                       "parallelism": f"points sharded x{world}, "
                                      f"{'RCCL' if args.transport == 'rccl' else 'host-staged (gloo)'} "
                                      f"all-reduce of {exchange}"},
            "device_ms_per_step": round(ms_dev, 4),
            "roofline": roofline,
            "iteration_roofline": iteration_roofline,
            "cpu_baseline": cpu,
            "mode": args.mode,
        }
        if trajectory is not None:
            out["trajectory"] = trajectory
        print(json.dumps(out), file=json_out, flush=True)
    solver.close()
    if host_ar is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
