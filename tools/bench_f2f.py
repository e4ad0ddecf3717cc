"""Frame-to-frame pose-only BA timing.

The reference solves every tracked frame with MotionOnlyBAOptimizerAngles
(Optimizer.cpp:417-457): 4 outer rounds of <= 20 LM iterations on one
6-vector over the frame's map-point correspondences.  This times ONE such
Ceres solve (max 20 iterations) three ways on synthetic frames of N
observations (make_synthetic motion-only mode):

  batch1   ba_solve_pose_batch with one frame (wall time, host round trip incl.)
  batchB   ba_solve_pose_batch with B frames in one launch (frames/s)
  solve    ba_set_problem + ba_solve (the general device path, per frame)
  cpu      the oracle's CPU restatement of Ceres LM (1 thread: the reference's
           motion-only problem is far below Ceres' threading threshold)

Prints one JSON line.  Usage: python tools/bench_f2f.py [--obs 500] [--batch 4096]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bundleadjustment_amd import Options, Solver, make_synthetic  # noqa: E402


def frames(n, n_obs, seed0):
    out = []
    for i in range(n):
        p = make_synthetic(1, n_obs, 1, seed=seed0 + i, motion_only=True)
        out.append(p)
    return out


def pack(problems):
    off = np.zeros(len(problems) + 1, np.int32)
    for i, p in enumerate(problems):
        off[i + 1] = off[i] + p.n_obs
    cams = np.array([p.cams[0] for p in problems])
    K = np.array([p.K[0] for p in problems])
    X = np.concatenate([p.pts[p.obs_pt] for p in problems])
    uv = np.concatenate([p.obs_uv for p in problems])
    return off, cams, K, X, uv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--obs", type=int, default=500)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    opts = Options(max_num_iterations=20)
    base = frames(64, a.obs, 0xF2F00000)
    res = dict(metric="frame-to-frame pose-only solve", obs_per_frame=float(np.mean([p.n_obs for p in base])),
               max_iterations=20)
    with Solver(0) as s:
        # batch of one frame: latency of one reference Ceres solve
        one = pack(base[:1])
        s.solve_pose_batch(*one, opts)
        t = []
        for r in range(a.reps):
            t0 = time.perf_counter()
            _, summ = s.solve_pose_batch(*pack(base[r % len(base):r % len(base) + 1]), opts)
            t.append(time.perf_counter() - t0)
        res["batch1_ms"] = 1e3 * float(np.median(t))
        res["batch1_lm_iterations"] = summ[0].num_iterations
        # general path per frame
        t = []
        for r in range(min(a.reps, 10)):
            p = base[r]
            t0 = time.perf_counter()
            s.set_problem(p)
            s.solve(opts)
            s.params()
            t.append(time.perf_counter() - t0)
        res["solve_ms"] = 1e3 * float(np.median(t))
        # large batch: throughput
        reps = (a.batch + len(base) - 1) // len(base)
        big = pack((base * reps)[:a.batch])
        s.solve_pose_batch(*big, opts)
        t = []
        for _ in range(3):
            t0 = time.perf_counter()
            _, summs = s.solve_pose_batch(*big, opts)
            t.append(time.perf_counter() - t0)
        tb = float(np.median(t))
        res["batch"] = a.batch
        res["batch_ms"] = 1e3 * tb
        res["batch_frames_per_s"] = a.batch / tb
        res["batch_mean_lm_iterations"] = float(np.mean([x.num_iterations for x in summs]))
    if not a.no_cpu:
        import oracle
        oracle.build()
        oracle.set_threads(1)
        t = []
        for p in base[:10]:
            t0 = time.perf_counter()
            oracle.solve(p, oracle.default_options(max_num_iterations=20))
            t.append(time.perf_counter() - t0)
        res["cpu_ms"] = 1e3 * float(np.median(t))
        res["cpu_kind"] = "port (oracle C++ restatement of Ceres LM, 1 thread), not Ceres"
        res["batch1_speedup_vs_cpu"] = res["cpu_ms"] / res["batch1_ms"]
        res["batch_speedup_vs_cpu"] = res["cpu_ms"] / (res["batch_ms"] / a.batch)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
