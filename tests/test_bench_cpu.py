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


# ---------------------------------------------------------------------------
# launch logic: `bench.py --gpus N` without a launcher starts its own N ranks
# (BA_BENCH_DRYRUN=1: every rank prints what it would run, no GPU call)
# ---------------------------------------------------------------------------
import json  # noqa: E402
import os  # noqa: E402
import subprocess  # noqa: E402


def _bench(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(BA_BENCH_DRYRUN="1", **env)
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True,
                          timeout=120, env=e)


def test_standalone_gpus_n_spawns_n_ranks():
    out = _bench(["--gpus", "4", "--steps", "7", "--warmup", "2"])
    assert out.returncode == 0, out.stderr
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.strip()]
    assert len(lines) == 1                      # rank 0's line only, relayed by the parent
    assert lines[0]["rank"] == 0 and lines[0]["world"] == 4 and lines[0]["device"] == 0
    assert lines[0]["workload"] == "c4"        # N > 1 default: BASELINE configs[3]
    assert lines[0]["steps"] == 7 and lines[0]["warmup"] == 2
    others = sorted(json.loads(x)["rank"] for x in out.stderr.splitlines() if x.startswith("{"))
    assert others == [1, 2, 3]
    devs = {json.loads(x)["rank"]: json.loads(x)["device"] for x in out.stderr.splitlines() if x.startswith("{")}
    assert devs == {1: 1, 2: 2, 3: 3}          # rank r on device r


def test_single_gpu_default_is_c3_without_spawning():
    out = _bench(["--gpus", "1"])
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout)
    assert d["world"] == 1 and d["workload"] == "c3"


def test_world_size_mismatch_is_an_error():
    out = _bench(["--gpus", "8"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr
    ok = _bench(["--gpus", "2"], WORLD_SIZE="2", RANK="1", LOCAL_RANK="1")   # under a launcher: one rank
    assert ok.returncode == 0 and json.loads(ok.stdout)["rank"] == 1


def test_failed_rank_fails_the_launch():
    out = _bench(["--gpus", "2"], BA_BENCH_DRYRUN_FAIL_RANK="1", BA_BENCH_DRYRUN_SLEEP="60")
    assert out.returncode == 3                 # the failing rank's status; the sleeping rank 0 is ended


def test_strong_workload_needs_a_divisor_of_8():
    out = _bench(["--gpus", "3", "--workload", "c4"])
    assert out.returncode != 0 and "dividing 8" in out.stderr


def test_host_transport_pins_the_device():
    out = _bench(["--gpus", "2", "--transport", "host", "--device", "0"])
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout)
    assert d["transport"] == "host" and d["device"] == 0
