"""Problem container (SoA, the C-ABI layout) and synthetic BAL-style problems.

Parameter layout is the reference's (ba_project/src/ba/Optimizer.h:54-76):
camera = [wx, wy, wz, tx, ty, tz] world->camera angle-axis + translation,
point = world XYZ; K float 3x3 column-major; fixed cameras carry a float 4x4
column-major world->camera extrinsic (PointOnlyReprojectionError,
Optimizer.h:96-107).

Synthetic problems follow SURVEY.md §8(d): seed 0xBA5E0000 + k, cameras on a
ring of radius 5 looking at the origin, points uniform in a ball of radius 2,
each point seen by exactly `obs_per_pt` cameras chosen uniformly among those
that see it in front of the camera and inside the image, 1 px Gaussian pixel
noise plus 5 % gross outliers, perturbed initial values, camera 0 anchored.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

HUBER_A = math.sqrt(5.991)  # ceres::HuberLoss(sqrt(5.991)), Optimizer.cpp:312

# Intrinsics hard-coded in the reference's VirtualSensor.h
FREIBURG = dict(fx=525.0, fy=525.0, cx=319.5, cy=239.5, w=640, h=480)   # VirtualSensor.h:160-162
REPLICA = dict(fx=600.0, fy=600.0, cx=599.5, cy=339.5, w=1200, h=680)   # VirtualSensor.h:112-114


@dataclass
class Problem:
    cams: np.ndarray                      # (C, 6) float64
    K: np.ndarray                         # (C, 9) float32, column-major
    pts: np.ndarray                       # (P, 3) float64
    obs_cam: np.ndarray                   # (N,) int32
    obs_pt: np.ndarray                    # (N,) int32
    obs_uv: np.ndarray                    # (N, 2) float32
    cam_fixed: np.ndarray | None = None   # (C,) uint8
    cam_fixed_extr: np.ndarray | None = None  # (C, 16) float32, column-major
    pt_fixed: np.ndarray | None = None    # (P,) uint8
    huber_a: float = HUBER_A
    gt_cams: np.ndarray | None = field(default=None, repr=False)
    gt_pts: np.ndarray | None = field(default=None, repr=False)
    name: str = ""

    @property
    def n_cams(self) -> int:
        return int(self.cams.shape[0])

    @property
    def n_pts(self) -> int:
        return int(self.pts.shape[0])

    @property
    def n_obs(self) -> int:
        return int(self.obs_cam.shape[0])

    def normalized(self) -> "Problem":
        """Contiguous arrays of the exact dtypes the C-ABI expects."""
        def c(a, dt, shape=None):
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=dt)
            return a.reshape(shape) if shape is not None else a
        return Problem(
            cams=c(self.cams, np.float64, (-1, 6)), K=c(self.K, np.float32, (-1, 9)),
            pts=c(self.pts, np.float64, (-1, 3)), obs_cam=c(self.obs_cam, np.int32),
            obs_pt=c(self.obs_pt, np.int32), obs_uv=c(self.obs_uv, np.float32, (-1, 2)),
            cam_fixed=c(self.cam_fixed, np.uint8), cam_fixed_extr=c(self.cam_fixed_extr, np.float32, (-1, 16)),
            pt_fixed=c(self.pt_fixed, np.uint8), huber_a=float(self.huber_a), gt_cams=self.gt_cams,
            gt_pts=self.gt_pts, name=self.name)

    def copy(self) -> "Problem":
        cp = lambda a: None if a is None else a.copy()
        return Problem(cp(self.cams), cp(self.K), cp(self.pts), cp(self.obs_cam), cp(self.obs_pt), cp(self.obs_uv),
                       cp(self.cam_fixed), cp(self.cam_fixed_extr), cp(self.pt_fixed), self.huber_a,
                       cp(self.gt_cams), cp(self.gt_pts), self.name)


# ---------------------------------------------------------------------------
# ceres rotation.h semantics, vectorised (column-major 3x3 as (..., 3, 3)
# standard matrices here: R[..., row, col]).
# ---------------------------------------------------------------------------
def angle_axis_to_rotation(w: np.ndarray) -> np.ndarray:
    """ceres::AngleAxisToRotationMatrix (first-order branch for theta^2 <= eps)."""
    w = np.asarray(w, dtype=np.float64)
    flat = w.reshape(-1, 3)
    th2 = np.einsum("ij,ij->i", flat, flat)
    R = np.empty((flat.shape[0], 3, 3))
    big = th2 > np.finfo(np.float64).eps
    if np.any(big):
        wb = flat[big]
        th = np.sqrt(th2[big])
        wx, wy, wz = (wb / th[:, None]).T
        c, s = np.cos(th), np.sin(th)
        oc = 1.0 - c
        R[big, 0, 0] = c + wx * wx * oc
        R[big, 1, 0] = wz * s + wx * wy * oc
        R[big, 2, 0] = -(wy * s) + wx * wz * oc
        R[big, 0, 1] = wx * wy * oc - wz * s
        R[big, 1, 1] = c + wy * wy * oc
        R[big, 2, 1] = wx * s + wy * wz * oc
        R[big, 0, 2] = wy * s + wx * wz * oc
        R[big, 1, 2] = -(wx * s) + wy * wz * oc
        R[big, 2, 2] = c + wz * wz * oc
    sm = ~big
    if np.any(sm):
        a = flat[sm]
        R[sm] = np.stack([np.stack([np.ones(len(a)), -a[:, 2], a[:, 1]], -1),
                          np.stack([a[:, 2], np.ones(len(a)), -a[:, 0]], -1),
                          np.stack([-a[:, 1], a[:, 0], np.ones(len(a))], -1)], 1)
    return R.reshape(w.shape[:-1] + (3, 3))


def rotation_to_angle_axis(R: np.ndarray) -> np.ndarray:
    """ceres::RotationMatrixToAngleAxis: Shepperd quaternion, then atan2."""
    R = np.asarray(R, dtype=np.float64)
    flat = R.reshape(-1, 3, 3)
    out = np.empty((flat.shape[0], 3))
    for n, M in enumerate(flat):
        q = [0.0, 0.0, 0.0, 0.0]
        tr = M[0, 0] + M[1, 1] + M[2, 2]
        if tr >= 0.0:
            t = math.sqrt(tr + 1.0)
            q[0] = 0.5 * t
            t = 0.5 / t
            q[1] = (M[2, 1] - M[1, 2]) * t
            q[2] = (M[0, 2] - M[2, 0]) * t
            q[3] = (M[1, 0] - M[0, 1]) * t
        else:
            i = 0
            if M[1, 1] > M[0, 0]:
                i = 1
            if M[2, 2] > M[i, i]:
                i = 2
            j, k = (i + 1) % 3, (i + 2) % 3
            t = math.sqrt(M[i, i] - M[j, j] - M[k, k] + 1.0)
            q[i + 1] = 0.5 * t
            t = 0.5 / t
            q[0] = (M[k, j] - M[j, k]) * t
            q[j + 1] = (M[j, i] + M[i, j]) * t
            q[k + 1] = (M[k, i] + M[i, k]) * t
        s2 = q[1] * q[1] + q[2] * q[2] + q[3] * q[3]
        if s2 > 0.0:
            st = math.sqrt(s2)
            ct = q[0]
            two = 2.0 * (math.atan2(-st, -ct) if ct < 0.0 else math.atan2(st, ct))
            kk = two / st
            out[n] = (q[1] * kk, q[2] * kk, q[3] * kk)
        else:
            out[n] = (q[1] * 2.0, q[2] * 2.0, q[3] * 2.0)
    return out.reshape(R.shape[:-2] + (3,))


def K_colmajor(fx, fy, cx, cy) -> np.ndarray:
    return np.array([fx, 0, 0, 0, fy, 0, cx, cy, 1], dtype=np.float32)


def extr_colmajor(R: np.ndarray, t: np.ndarray) -> np.ndarray:
    E = np.eye(4, dtype=np.float32)
    E[:3, :3] = R.astype(np.float32)
    E[:3, 3] = t.astype(np.float32)
    return E.T.reshape(16).copy()   # column-major flatten


def project(R: np.ndarray, t: np.ndarray, K9: np.ndarray, X: np.ndarray) -> np.ndarray:
    """Pinhole projection of points X (N,3) with per-row R (N,3,3), t (N,3), K (N,9) col-major."""
    p = np.einsum("nij,nj->ni", R, X) + t
    Kd = K9.astype(np.float64).reshape(-1, 3, 3).transpose(0, 2, 1)
    q = np.einsum("nij,nj->ni", Kd, p)
    return q[:, :2] / q[:, 2:3], p[:, 2]


# ---------------------------------------------------------------------------
# synthetic problems
# ---------------------------------------------------------------------------
CONFIGS = {
    # name: (cams, points, obs/pt, intrinsics, motion_only)
    "f2f": dict(n_cams=1, n_pts=500, obs_per_pt=1, intr="freiburg", motion_only=True),
    "c1": dict(n_cams=2, n_pts=500, obs_per_pt=2, intr="freiburg"),
    "c2": dict(n_cams=50, n_pts=10_000, obs_per_pt=5, intr="replica"),
    "c3": dict(n_cams=200, n_pts=100_000, obs_per_pt=10, intr="freiburg"),
    "c4": dict(n_cams=1_000, n_pts=1_000_000, obs_per_pt=10, intr="freiburg"),
    "c5": dict(n_cams=10_000, n_pts=10_000_000, obs_per_pt=10, intr="freiburg"),
}
CONFIG_INDEX = {"f2f": 0, "c1": 0, "c2": 1, "c3": 2, "c4": 3, "c5": 4}


def _look_at(center: np.ndarray, target: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    z = target - center
    z /= np.linalg.norm(z)
    up = np.array([0.0, 0.0, 1.0])
    x = np.cross(z, up)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z])           # rows = camera axes in world: world->camera
    return R, -R @ center


def make_synthetic(n_cams: int, n_pts: int, obs_per_pt: int = 10, seed: int = 0xBA5E0002,
                   intr: str = "freiburg", noise_px: float = 1.0, outlier_frac: float = 0.05,
                   perturb=(0.01, 0.02, 0.02), anchor: bool = True, motion_only: bool = False,
                   name: str = "", point_seed: int | None = None) -> Problem:
    """`seed` drives the cameras (and their initial perturbation); `point_seed`
    (default: same stream) drives points, visibility, pixel noise and point
    perturbation — so point shards of one scene share identical cameras."""
    rng = np.random.default_rng(seed)
    I = FREIBURG if intr == "freiburg" else REPLICA
    W, H = I["w"], I["h"]
    K9 = K_colmajor(I["fx"], I["fy"], I["cx"], I["cy"])
    Kf = np.tile(K9, (n_cams, 1))
    # cameras on a ring of radius 5 (height jitter) looking at the origin
    if n_cams == 1:
        phis = np.array([0.0])
    else:
        phis = np.linspace(0.0, 2.0 * np.pi, n_cams, endpoint=False)
    Rs = np.empty((n_cams, 3, 3))
    ts = np.empty((n_cams, 3))
    for i, ph in enumerate(phis):
        h = rng.uniform(-1.0, 1.0) if n_cams > 2 else 0.3 * i
        if n_cams == 2:
            ph = 0.25 * i
        center = np.array([5.0 * np.cos(ph), 5.0 * np.sin(ph), h])
        target = rng.normal(0.0, 0.1, 3)
        Rs[i], ts[i] = _look_at(center, target)
    cam_noise = None
    if perturb is not None:
        cam_noise = (rng.normal(0.0, perturb[0], size=(n_cams, 3)), rng.normal(0.0, perturb[1], size=(n_cams, 3)))
    if point_seed is not None:
        rng = np.random.default_rng(point_seed)
    # points uniform in a ball of radius 2
    d = rng.normal(size=(n_pts, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    X = d * (2.0 * rng.uniform(size=(n_pts, 1)) ** (1.0 / 3.0))
    k = min(obs_per_pt, n_cams)
    # visibility-constrained uniform choice of k cameras per point
    m = n_cams if n_cams <= 512 else min(n_cams, 8 * k + 64)
    obs_c, obs_p = [], []
    chunk = max(1, 4_000_000 // max(m, 1))
    for s0 in range(0, n_pts, chunk):
        Xc = X[s0:s0 + chunk]
        nb = Xc.shape[0]
        cand = (np.tile(np.arange(n_cams), (nb, 1)) if m == n_cams
                else rng.integers(0, n_cams, size=(nb, m)))
        Rc, tc = Rs[cand], ts[cand]                                     # (nb, m, 3, 3)
        pc = np.einsum("bmij,bj->bmi", Rc, Xc) + tc
        z = pc[..., 2]
        u = I["fx"] * pc[..., 0] / z + I["cx"]
        v = I["fy"] * pc[..., 1] / z + I["cy"]
        vis = (z > 0.1) & (u >= 0) & (u < W) & (v >= 0) & (v < H)
        if m != n_cams:  # de-duplicate sampled candidates
            srt = np.sort(cand, axis=1)
            dup = np.zeros_like(vis)
            order = np.argsort(cand, axis=1, kind="stable")
            dup_sorted = np.concatenate([np.zeros((nb, 1), bool), srt[:, 1:] == srt[:, :-1]], 1)
            np.put_along_axis(dup, order, dup_sorted, axis=1)
            vis &= ~dup
        key = rng.uniform(size=vis.shape)
        key[~vis] = 2.0
        sel = np.argsort(key, axis=1)[:, :k]
        ok = np.take_along_axis(key, sel, 1) < 2.0
        cams_sel = np.take_along_axis(cand, sel, 1)
        cams_sel = np.where(ok, cams_sel, -1)
        cams_sel.sort(axis=1)
        pid = np.repeat(np.arange(s0, s0 + nb)[:, None], k, 1)
        keep = cams_sel >= 0
        obs_c.append(cams_sel[keep])
        obs_p.append(pid[keep])
    obs_cam = np.concatenate(obs_c).astype(np.int32)
    obs_pt = np.concatenate(obs_p).astype(np.int32)
    # drop points with fewer than 2 observations (unless motion-only)
    if not motion_only:
        cnt = np.bincount(obs_pt, minlength=n_pts)
        good = cnt[obs_pt] >= min(2, k)
        obs_cam, obs_pt = obs_cam[good], obs_pt[good]
    uv, _ = project(Rs[obs_cam], ts[obs_cam], Kf[obs_cam], X[obs_pt])
    n_obs = len(obs_cam)
    if noise_px > 0:
        uv = uv + rng.normal(0.0, noise_px, size=uv.shape)
    if outlier_frac > 0:
        bad = rng.uniform(size=n_obs) < outlier_frac
        uv[bad, 0] = rng.uniform(0, W, size=bad.sum())
        uv[bad, 1] = rng.uniform(0, H, size=bad.sum())
    w_gt = rotation_to_angle_axis(Rs)
    gt_cams = np.concatenate([w_gt, ts], 1)
    cams = gt_cams.copy()
    pts = X.copy()
    if perturb is not None:
        cams[:, :3] += cam_noise[0]
        cams[:, 3:] += cam_noise[1]
        if not motion_only:
            pts += rng.normal(0.0, perturb[2], size=pts.shape)
    cam_fixed = np.zeros(n_cams, np.uint8)
    extr = np.zeros((n_cams, 16), np.float32)
    if anchor and not motion_only:
        cam_fixed[0] = 1
        extr[0] = extr_colmajor(Rs[0], ts[0])
        # the anchor's angle-axis is what prepareConstraints derives from the
        # float extrinsic (Optimizer.cpp:296-299)
        Rf = extr[0].reshape(4, 4).T[:3, :3].astype(np.float64)
        cams[0, :3] = rotation_to_angle_axis(Rf)
        cams[0, 3:] = extr[0].reshape(4, 4).T[:3, 3].astype(np.float64)
    pt_fixed = None
    if motion_only:
        pt_fixed = np.ones(n_pts, np.uint8)
        pts = pts.astype(np.float32).astype(np.float64)   # Vector4f homogeneous point (Optimizer.h:158)
    return Problem(cams=cams, K=Kf, pts=pts, obs_cam=obs_cam, obs_pt=obs_pt, obs_uv=uv.astype(np.float32),
                   cam_fixed=cam_fixed, cam_fixed_extr=extr, pt_fixed=pt_fixed, huber_a=HUBER_A,
                   gt_cams=gt_cams, gt_pts=X, name=name).normalized()


def fix_camera(problem: Problem, c: int) -> Problem:
    """Anchor camera c at its current estimate the way prepareConstraints does
    for keyframe 0 (Optimizer.cpp:296-299, 314-321): the constant functor gets
    the float 4x4 extrinsic, the angle-axis block is re-derived from it."""
    R = angle_axis_to_rotation(problem.cams[c, :3])
    if problem.cam_fixed is None:
        problem.cam_fixed = np.zeros(problem.n_cams, np.uint8)
    if problem.cam_fixed_extr is None:
        problem.cam_fixed_extr = np.zeros((problem.n_cams, 16), np.float32)
    problem.cam_fixed[c] = 1
    problem.cam_fixed_extr[c] = extr_colmajor(R, problem.cams[c, 3:])
    E = problem.cam_fixed_extr[c].reshape(4, 4).T
    problem.cams[c, :3] = rotation_to_angle_axis(E[:3, :3].astype(np.float64))
    problem.cams[c, 3:] = E[:3, 3].astype(np.float64)
    return problem


def make_config(name: str, scale: float = 1.0, **overrides) -> Problem:
    """Synthetic problem of a BASELINE.json config (seed 0xBA5E0000 + config index)."""
    cfg = dict(CONFIGS[name])
    cfg.update(overrides)
    if scale != 1.0:
        cfg["n_pts"] = max(1, int(cfg["n_pts"] * scale))
    seed = cfg.pop("seed", 0xBA5E0000 + CONFIG_INDEX[name])
    return make_synthetic(seed=seed, name=name, **cfg)


def shard_points(problem: Problem, nranks: int, rank: int, bounds: list[int] | None = None) -> Problem:
    """Point-sharded slice for multi-GPU: contiguous point
    ranges balanced by observation count (or the given `bounds`, nranks + 1
    point offsets; a rank may get none); cameras replicated; the shard keeps
    only its points' observations (re-indexed)."""
    bounds = shard_bounds(problem, nranks) if bounds is None else bounds
    p0, p1 = bounds[rank], bounds[rank + 1]
    sel = (problem.obs_pt >= p0) & (problem.obs_pt < p1)
    sub = problem.copy()
    sub.pts = problem.pts[p0:p1].copy()
    sub.pt_fixed = None if problem.pt_fixed is None else problem.pt_fixed[p0:p1].copy()
    sub.obs_cam = problem.obs_cam[sel].copy()
    sub.obs_pt = (problem.obs_pt[sel] - p0).astype(np.int32)
    sub.obs_uv = problem.obs_uv[sel].copy()
    sub.gt_pts = None if problem.gt_pts is None else problem.gt_pts[p0:p1].copy()
    return sub.normalized()


def shard_bounds(problem: Problem, nranks: int) -> list[int]:
    cnt = np.bincount(problem.obs_pt, minlength=problem.n_pts).astype(np.int64)
    csum = np.concatenate([[0], np.cumsum(cnt)])
    total = csum[-1]
    b = [int(np.searchsorted(csum, total * r / nranks, side="left")) for r in range(nranks + 1)]
    b[0], b[-1] = 0, problem.n_pts
    return b
