"""The multi-rank LM iteration of libba_hip on hardware: 2 and 3 ranks, each
a separate process with its own ba_ctx on the one GPU of the box, points
sharded, cameras replicated.  RCCL refuses
several ranks on one device, so the exchange goes through the host-staged
transport (ba_comm_init_host -> torch.distributed gloo); every all-reduce of
the LM iteration (camera blocks, gradient norms, the packed reduced system
or the folded CG matvec, the step scalars) runs exactly as with RCCL, only
the transport differs.

The sharded solve must reproduce the single-process solve of the whole
problem: identical accept/reject decisions and CG counts, costs 1e-9,
cameras (replicated: bitwise equal across ranks) and each rank's points 1e-8.
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from bundleadjustment_amd import Options, make_config, make_synthetic
from bundleadjustment_amd.problem import fix_camera, shard_bounds

ROOT = Path(__file__).resolve().parents[1]


def scene(name="c2"):
    # gauge-fixed (two anchors): one isolated minimum, trajectories comparable.
    # "many": more cameras than the LDS camera table holds (> kLinLdsCams),
    # so the compact-record linearisation, the global camera tables and the
    # JR records with the residual copy run through the exchange path
    if name == "many":
        return fix_camera(make_synthetic(300, 12_000, 6, seed=0xBA5E0011), 1)
    if name == "empty":
        return fix_camera(make_config("c2", scale=0.25), 1)
    return fix_camera(make_config("c2", scale=0.5), 1)


def scene_bounds(p, world, name):
    """Point offsets of the ranks' shards: balanced, or for "empty" every
    point on rank 0 and none on the others (a rank with no observations: the
    clamped-index prologues of k_obs_w & co. and the max_no choice)."""
    if name == "empty":
        return [0] + [p.n_pts] * world
    return shard_bounds(p, world)


def solve_options(lin, prec):
    return Options(max_num_iterations=8, linear_solver_type=lin, preconditioner_type="SCHUR_JACOBI", precision=prec)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("lin,prec", [("DENSE_SCHUR", "FP64"), ("ITERATIVE_SCHUR", "FP64"),
                                      ("ITERATIVE_SCHUR", "MIXED_FP32")])
def test_sharded_solve_matches_single_rank(tmp_path, world, lin, prec):
    run_sharded(tmp_path, world, lin, prec, "c2")


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("lin", ["DENSE_SCHUR", "ITERATIVE_SCHUR"])
def test_sharded_many_cameras_matches_single_rank(tmp_path, lin):
    run_sharded(tmp_path, 2, lin, "FP64", "many")


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("lin,prec", [("DENSE_SCHUR", "FP64"), ("ITERATIVE_SCHUR", "FP64"),
                                      ("ITERATIVE_SCHUR", "MIXED_FP32")])
def test_sharded_solve_with_an_empty_rank(tmp_path, lin, prec):
    run_sharded(tmp_path, 2, lin, prec, "empty")


def run_sharded(tmp_path, world, lin, prec, name):
    from bundleadjustment_amd import Solver
    p = scene(name)
    with Solver(0) as s:
        s.set_problem(p)
        ref = s.solve(solve_options(lin, prec))
        rc, rp = s.params()
        rlog = s.iteration_log()
    port = str(free_port())
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([str(ROOT / "tests"), str(ROOT)]))
    procs = [subprocess.Popen([sys.executable, str(ROOT / "tests" / "mr_worker.py"), str(r), str(world), port,
                               str(tmp_path), lin, prec, name], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT,
                              text=True) for r in range(world)]
    outs = []
    for pr in procs:
        try:
            outs.append(pr.communicate(timeout=300)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(pr.returncode == 0 for pr in procs), "\n".join(outs)
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    bounds = scene_bounds(p, world, name)
    for r, d in enumerate(res):
        assert np.array_equal(d["cams"], res[0]["cams"])          # replicated, identical decisions
        assert d["ok"].tolist() == [x["step_is_successful"] for x in rlog]
        assert d["cg"].tolist() == [x["linear_solver_iterations"] for x in rlog]
        np.testing.assert_allclose(d["cost"], [x["cost"] for x in rlog], rtol=1e-9)
        np.testing.assert_allclose(d["pts"], rp[bounds[r]:bounds[r + 1]], rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(res[0]["cams"], rc, rtol=1e-8, atol=1e-10)
    assert float(res[0]["final"]) == pytest.approx(ref.final_cost, rel=1e-9)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_gpus_2_launches_its_ranks(tmp_path):
    """`bench.py --gpus 2` without a launcher starts both ranks itself and
    reports the 2-rank C4 strong-scaling line (host-staged transport: both
    ranks share the box's one GPU)."""
    import json
    sys.path.insert(0, str(ROOT))
    import bench
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--workload", "c4", "--scale",
                          "0.02", "--steps", "3", "--warmup", "1", "--transport", "host", "--device", "0",
                          "--no-cpu-baseline"], capture_output=True, text=True, timeout=500, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    whole = bench.strong_shard("c4", 0, 1, 0.02)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["steps"] == 3
    assert d["config"]["global_obs"] == whole.n_obs
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert abs(d["value"] - whole.n_obs * 3 / (d["ms_per_step"] * 3e-3) / 1e6) <= 0.01 * d["value"]
