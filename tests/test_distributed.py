"""Multi-GPU decomposition, checked on CPU with torch.distributed (gloo,
world_size 2, 127.0.0.1).

The RCCL path of libba_hip shards points
across ranks, keeps cameras replicated, and all-reduces the camera column
norms (Jacobi scaling), the camera blocks and the dense reduced camera
system.  That is only correct if the reduced system is a sum over point
shards plus the camera LM diagonal once.  Here two gloo ranks compute their
shard's contribution with the oracle, all-reduce it, and must reproduce the
unsharded system and step.  The rendezvous of bench.py (RCCL id through a
launcher-keyed file) is exercised with two processes as well.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from bundleadjustment_amd import make_synthetic
from bundleadjustment_amd.problem import fix_camera, shard_bounds, shard_points

WORLD = 2


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def scene():
    # every camera is observed from both halves of the points
    return fix_camera(make_synthetic(24, 3000, 6, seed=21), 1)


def _shard_worker(rank, port, out_dir):
    import torch

    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        oracle.set_threads(2)
        p = scene()
        local = shard_points(p, WORLD, rank)
        cn = torch.from_numpy(oracle.camera_colnorm2(local))
        dist.all_reduce(cn)                                   # ~ RCCL all-reduce of Hcc diagonals
        lhs, rhs = oracle.reduced_system(local, cam_colnorm2=cn.numpy(), add_cam_D=(rank == 0))
        L, R = torch.from_numpy(lhs), torch.from_numpy(rhs)
        dist.all_reduce(L)                                    # ~ RCCL all-reduce of S
        dist.all_reduce(R)
        if rank == 0:
            np.savez(os.path.join(out_dir, "sharded.npz"), lhs=L.numpy(), rhs=R.numpy(), cn=cn.numpy())
    finally:
        dist.destroy_process_group()


def test_reduced_system_is_a_sum_over_point_shards(tmp_path, oracle_lib):
    p = scene()
    b = shard_bounds(p, WORLD)
    assert b[0] == 0 and b[-1] == p.n_pts and b[0] < b[1] < b[2]
    mp.spawn(_shard_worker, args=(free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    got = np.load(tmp_path / "sharded.npz")
    lhs, rhs = oracle_lib.reduced_system(p)
    assert got["lhs"].shape == lhs.shape
    tril = np.tril_indices(lhs.shape[0])
    scale = np.abs(lhs[tril]).max()
    assert np.allclose(got["lhs"][tril], lhs[tril], rtol=1e-12, atol=1e-13 * scale)
    assert np.allclose(got["rhs"], rhs, rtol=1e-12, atol=1e-13 * np.abs(rhs).max())
    assert np.allclose(got["cn"].reshape(-1, 6), oracle_lib.camera_colnorm2(p), rtol=1e-13)
    # the camera step of both systems
    full = np.tril(lhs) + np.tril(lhs, -1).T
    shd = np.tril(got["lhs"]) + np.tril(got["lhs"], -1).T
    y_full = np.linalg.solve(full, rhs)
    y_shd = np.linalg.solve(shd, got["rhs"])
    assert np.allclose(y_shd, y_full, rtol=1e-9, atol=1e-12 * np.abs(y_full).max())


def _rendezvous_worker(rank, port, out_dir):
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from bundleadjustment_amd import Solver
    Solver.unique_id = staticmethod(lambda: bytes(range(128)))   # no RCCL needed to test the protocol
    uid = bench.rendezvous_uid(rank, WORLD, timeout_s=60)
    with open(os.path.join(out_dir, f"uid{rank}.bin"), "wb") as f:
        f.write(uid)


def test_bench_rendezvous_shares_the_rccl_id(tmp_path):
    port = free_port()
    mp.spawn(_rendezvous_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True)
    ids = [(tmp_path / f"uid{r}.bin").read_bytes() for r in range(WORLD)]
    assert ids[0] == ids[1] == bytes(range(128))


@pytest.mark.parametrize("n", [2, 3, 8])
def test_shards_partition_points_and_observations(n):
    p = make_synthetic(10, 1000, 4, seed=5)
    shards = [shard_points(p, n, r) for r in range(n)]
    assert sum(s.n_pts for s in shards) == p.n_pts
    assert sum(s.n_obs for s in shards) == p.n_obs
    counts = [s.n_obs for s in shards]
    assert max(counts) - min(counts) <= 2 * 4          # balanced by observation count
    for s in shards:
        assert np.array_equal(s.cams, p.cams)          # cameras replicated
