"""bench.py host logic (CPU): the strong-scaling workloads split ONE fixed
global problem — the union of the rank shards is the same problem for every
rank count that divides the 8 point blocks."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def _union(cfg, world):
    parts = [bench.strong_shard(cfg, r, world) for r in range(world)]
    pts = np.concatenate([p.pts for p in parts])
    obs = np.concatenate([np.column_stack([p.obs_cam, p.pts[p.obs_pt]]) for p in parts])
    order = np.lexsort(pts.T[::-1])
    oorder = np.lexsort(obs.T[::-1])
    return parts, pts[order], obs[oorder]


def test_strong_shards_partition_one_problem(monkeypatch):
    # the c3 generator with 8 blocks keeps this fast; c4 / c5 use the same code
    monkeypatch.setitem(bench.STRONG, "c3", dict(blocks=8, solver="ITERATIVE_SCHUR", precision="FP64"))
    p1, pts1, obs1 = _union("c3", 1)
    for world in (2, 4, 8):
        pw, ptsw, obsw = _union("c3", world)
        assert np.array_equal(pts1, ptsw) and np.array_equal(obs1, obsw)
        for p in pw:   # every rank keeps all cameras (replicated), identical values
            assert np.array_equal(p.cams, p1[0].cams) and p.n_cams == p1[0].n_cams
    assert p1[0].n_pts == 8 * (100_000 // 8)
