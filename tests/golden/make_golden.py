"""Generate tests/golden/functors.npz — golden residuals and Jacobians of the
reference's three cost functors (ba_project/src/ba/Optimizer.h:49-194).

Independent restatement in torch fp64, differentiated by torch.func.jacfwd
(forward-mode AD, the same mechanism as ceres::AutoDiffCostFunction).  The
reference itself cannot run here (Ceres/Eigen absent), so these vectors pin
the oracle and the HIP kernels to one another, not to Ceres: parity with the
reference remains "unpinned" (DESIGN.md §5).

Run:  python tests/golden/make_golden.py     (CPU only, a few seconds)
"""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np
import torch
from torch.func import jacfwd

torch.set_default_dtype(torch.float64)
EPS = np.finfo(np.float64).eps


def angle_axis_to_R(w: torch.Tensor) -> torch.Tensor:
    """ceres::AngleAxisToRotationMatrix, returns R[row, col]."""
    th2 = w @ w
    if float(th2) > EPS:
        th = torch.sqrt(th2)
        wx, wy, wz = w[0] / th, w[1] / th, w[2] / th
        c, s = torch.cos(th), torch.sin(th)
        oc = 1.0 - c
        return torch.stack([
            torch.stack([c + wx * wx * oc, wx * wy * oc - wz * s, wy * s + wx * wz * oc]),
            torch.stack([wz * s + wx * wy * oc, c + wy * wy * oc, -(wx * s) + wy * wz * oc]),
            torch.stack([-(wy * s) + wx * wz * oc, wx * s + wy * wz * oc, c + wz * wz * oc]),
        ])
    one = torch.ones((), dtype=w.dtype)
    return torch.stack([torch.stack([one, -w[2], w[1]]), torch.stack([w[2], one, -w[0]]),
                        torch.stack([-w[1], w[0], one])])


def proj(K, p, uv):
    q = K @ p
    return q[:2] / q[2] - uv


def angle_reprojection(cam, pt, K, uv):           # Optimizer.h:54-76
    R = angle_axis_to_R(cam[:3])
    return proj(K, R @ pt + cam[3:], uv)


def point_only(pt, E, K, uv):                      # Optimizer.h:96-107
    ph = E @ torch.cat([pt, torch.ones(1)])
    return proj(K, ph[:3] / ph[3], uv)


def pose_only(cam, X, K, uv):                      # Optimizer.h:163-182
    R = angle_axis_to_R(cam[:3])
    return proj(K, R @ X + cam[3:], uv)


def main(out: Path):
    rng = np.random.default_rng(20260115)
    Kf = np.array([[525, 0, 319.5], [0, 525, 239.5], [0, 0, 1]], np.float32)
    Kr = np.array([[600, 0, 599.5], [0, 600, 339.5], [0, 0, 1]], np.float32)
    n = 256
    kinds = {"generic": lambda: rng.normal(0, 0.6, 3),
             "small": lambda: rng.normal(0, 1, 3) * 1e-9,          # theta^2 <= DBL_EPSILON branch
             "zero": lambda: np.zeros(3),
             "near_pi": lambda: (lambda a: a / np.linalg.norm(a) * (math.pi - abs(rng.normal(0, 1e-3))))(
                 rng.normal(size=3)),
             "threshold": lambda: (lambda a: a / np.linalg.norm(a) * math.sqrt(EPS) * rng.uniform(0.5, 2.0))(
                 rng.normal(size=3))}
    cams, pts, Ks, uvs, kind_id = [], [], [], [], []
    for ki, (name, gen) in enumerate(kinds.items()):
        for _ in range(n):
            w = gen()
            t = rng.normal(0, 0.5, 3) + np.array([0, 0, 5.0])
            X = rng.normal(0, 1.0, 3)
            K = Kf if rng.uniform() < 0.5 else Kr
            uv = rng.uniform([0, 0], [640, 480]).astype(np.float32)
            cams.append(np.concatenate([w, t])); pts.append(X); Ks.append(K.T.reshape(9)); uvs.append(uv)
            kind_id.append(ki)
    cams = np.array(cams); pts = np.array(pts); Ks = np.array(Ks, np.float32); uvs = np.array(uvs, np.float32)
    m = len(cams)
    r_angle = np.empty((m, 2)); J_angle = np.empty((m, 2, 9))
    r_pose = np.empty((m, 2)); J_pose = np.empty((m, 2, 6))
    r_pt = np.empty((m, 2)); J_pt = np.empty((m, 2, 3))
    extr = np.empty((m, 16), np.float32)
    for i in range(m):
        K = torch.tensor(Ks[i].reshape(3, 3).T.astype(np.float64))
        uv = torch.tensor(uvs[i].astype(np.float64))
        c = torch.tensor(cams[i]); X = torch.tensor(pts[i])
        f = lambda cp: angle_reprojection(cp[:6], cp[6:], K, uv)
        x = torch.cat([c, X])
        r_angle[i] = f(x).numpy(); J_angle[i] = jacfwd(f)(x).numpy()
        Xf = torch.tensor(pts[i].astype(np.float32).astype(np.float64))
        g = lambda cc: pose_only(cc, Xf, K, uv)
        r_pose[i] = g(c).numpy(); J_pose[i] = jacfwd(g)(c).numpy()
        R = angle_axis_to_R(c[:3]).numpy()
        E = np.eye(4, dtype=np.float32); E[:3, :3] = R; E[:3, 3] = cams[i][3:]
        extr[i] = E.T.reshape(16)
        Et = torch.tensor(E.astype(np.float64))
        h = lambda pp: point_only(pp, Et, K, uv)
        r_pt[i] = h(X).numpy(); J_pt[i] = jacfwd(h)(X).numpy()
    np.savez_compressed(out, cams=cams, pts=pts, K=Ks, uv=uvs, kind=np.array(kind_id, np.int32),
                        kind_names=np.array(list(kinds)), extr=extr, r_angle=r_angle, J_angle=J_angle,
                        r_pose=r_pose, J_pose=J_pose, r_pt=r_pt, J_pt=J_pt)
    print(f"wrote {out} ({m} cases)")


if __name__ == "__main__":
    main(Path(__file__).resolve().parent / "functors.npz")
