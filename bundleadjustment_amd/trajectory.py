"""Trajectory output and absolute trajectory error.

* ``write_tum_trajectory`` restates the reference's keyframe trajectory
  writer (ba_project/src/ba/BundleAdjustment.cpp:249-268): one line per
  keyframe, ``stamp tx ty tz qx qy qz qw`` of the camera->world pose
  (``Frame::getPose``), ``std::fixed`` with 4 decimals, the quaternion from
  Eigen's ``Quaternionf(Matrix3f)`` in float.  (Eigen is unpinned and absent
  here; ``quaternion_from_rotation`` restates its published branch structure:
  trace > 0 -> w from the trace, else the largest diagonal element.)  Note
  the reference's 4-decimal output: trajectories it writes are quantised to
  0.1 mm, which bounds any ATE comparison made from its files.
* ``read_file_list`` / ``associate`` / ``align`` / ``ate`` restate the TUM
  tools the reference evaluates with (src/metrics/associate.py:50-110,
  src/metrics/evaluate_ate_scale.py:51-97 and :150-175): greedy timestamp
  association within ``max_difference``, Horn's closed-form rotation from
  the SVD of the centred cross-covariance with the reflection fix, the
  least-squares scale  s = sum <d_i, R m_i> / sum |m_i|^2, and the RMSE /
  mean / median / std / min / max of the aligned translational error.
  Pinned against the reference script itself: tests/golden/ate.json
  (made by tests/golden/make_ate_golden.py in the build container).
"""
from __future__ import annotations

import math
import os

import numpy as np


# ---------------------------------------------------------------------------
# writer
# ---------------------------------------------------------------------------
def quaternion_from_rotation(R: np.ndarray) -> tuple[float, float, float, float]:
    """Eigen QuaternionBase::operator=(MatrixBase) for a float 3x3 (x, y, z, w)."""
    m = np.asarray(R, dtype=np.float32)
    f = np.float32
    t = f(m[0, 0] + m[1, 1] + m[2, 2])
    q = [f(0), f(0), f(0), f(0)]   # x, y, z, w
    if t > f(0):
        t = f(np.sqrt(f(t + f(1))))
        q[3] = f(f(0.5) * t)
        t = f(f(0.5) / t)
        q[0] = f(f(m[2, 1] - m[1, 2]) * t)
        q[1] = f(f(m[0, 2] - m[2, 0]) * t)
        q[2] = f(f(m[1, 0] - m[0, 1]) * t)
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = f(np.sqrt(f(f(f(m[i, i] - m[j, j]) - m[k, k]) + f(1))))
        q[i] = f(f(0.5) * t)
        t = f(f(0.5) / t)
        q[3] = f(f(m[k, j] - m[j, k]) * t)
        q[j] = f(f(m[j, i] + m[i, j]) * t)
        q[k] = f(f(m[k, i] + m[i, k]) * t)
    return tuple(float(v) for v in q)


def write_tum_trajectory(path: str | os.PathLike, stamps, poses) -> None:
    """Keyframe trajectory as the reference writes it (BundleAdjustment.cpp:252-266).

    stamps: (N,) timestamps; poses: (N, 4, 4) camera->world (row-major
    matrices, i.e. ``Frame::getPose()``), stored as float like Matrix4f."""
    poses = np.asarray(poses, dtype=np.float32).reshape(-1, 4, 4)
    with open(path, "w") as f:
        for s, P in zip(stamps, poses):
            qx, qy, qz, qw = quaternion_from_rotation(P[:3, :3])
            tx, ty, tz = (float(v) for v in P[:3, 3])
            f.write(f"{float(s):.4f} {tx:.4f} {ty:.4f} {tz:.4f} {qx:.4f} {qy:.4f} {qz:.4f} {qw:.4f}\n")


# ---------------------------------------------------------------------------
# evaluation
# ---------------------------------------------------------------------------
def read_file_list(path: str | os.PathLike) -> dict[float, list[str]]:
    """``stamp d1 d2 ...`` lines (',' and tabs as separators, '#' comments)."""
    out: dict[float, list[str]] = {}
    with open(path) as f:
        text = f.read().replace(",", " ").replace("\t", " ")
    for line in text.split("\n"):
        if not line or line[0] == "#":
            continue
        fields = [v for v in line.split(" ") if v.strip()]
        if len(fields) > 1:
            out[float(fields[0])] = fields[1:]
    return out


def associate(first: dict, second: dict, offset: float = 0.0, max_difference: float = 0.02) -> list[tuple]:
    """Greedy one-to-one matching by ascending |a - (b + offset)| < max_difference,
    returned sorted by the first stamp (ties broken by (a, b) like the
    reference's sorted() of (diff, a, b) triples)."""
    a = np.array(sorted(first), dtype=np.float64)
    b = np.array(sorted(second), dtype=np.float64)
    if a.size == 0 or b.size == 0:
        return []
    cands = []
    # windowed candidate search (the reference scans all pairs; same set)
    lo = np.searchsorted(b + offset, a - max_difference, side="left")
    hi = np.searchsorted(b + offset, a + max_difference, side="right")
    for ia in range(a.size):
        for ib in range(lo[ia], hi[ia]):
            d = abs(a[ia] - (b[ib] + offset))
            if d < max_difference:
                cands.append((d, a[ia], b[ib]))
    cands.sort()
    used_a, used_b, matches = set(), set(), []
    for _, x, y in cands:
        if x not in used_a and y not in used_b:
            used_a.add(x)
            used_b.add(y)
            matches.append((x, y))
    matches.sort()
    return matches


def align(model: np.ndarray, data: np.ndarray):
    """Similarity alignment of ``model`` (3, n) onto ``data`` (3, n):
    returns (R, t, per-point error, s) with data ~ s R model + t."""
    model = np.asarray(model, np.float64)
    data = np.asarray(data, np.float64)
    mc = model - model.mean(1, keepdims=True)
    dc = data - data.mean(1, keepdims=True)
    W = mc @ dc.T                                   # sum of outer(m_i, d_i)
    U, _, Vh = np.linalg.svd(W.T)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vh) < 0:
        S[2, 2] = -1.0
    R = U @ S @ Vh
    rm = R @ mc
    s = float(np.sum(dc * rm) / np.sum(mc * mc))
    t = data.mean(1, keepdims=True) - s * (R @ model.mean(1, keepdims=True))
    err = np.sqrt(np.sum((s * (R @ model) + t - data) ** 2, 0))
    return R, t, err, s


def ate(gt_path, est_path, offset: float = 0.0, scale: float = 1.0, max_difference: float = 0.02) -> dict:
    """evaluate_ate_scale.py's numbers for two TUM trajectory files."""
    first = read_file_list(gt_path)
    second = read_file_list(est_path)
    matches = associate(first, second, offset, max_difference)
    if len(matches) < 2:
        raise ValueError("couldn't find matching timestamp pairs between groundtruth and estimated trajectory")
    gt = np.array([[float(v) for v in first[a][0:3]] for a, _ in matches]).T
    est = np.array([[float(v) * scale for v in second[b][0:3]] for _, b in matches]).T
    R, t, err, s = align(est, gt)
    return dict(pairs=len(matches), rmse=math.sqrt(float(np.dot(err, err)) / len(err)), mean=float(np.mean(err)),
                median=float(np.median(err)), std=float(np.std(err)), min=float(np.min(err)),
                max=float(np.max(err)), scale=s, rot=R, trans=t.reshape(3), matches=matches)
