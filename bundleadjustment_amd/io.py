"""Problem I/O: BAL text format and the binary SoA dump.

Two exchange formats for problems in the reference's parameter layout
(camera = [wx, wy, wz, tx, ty, tz] world->camera angle-axis + translation,
Optimizer.h:54-76; K float 3x3 column-major; fixed cameras carry a float 4x4
column-major extrinsic, Optimizer.h:96-107):

* **BAS dump** (``save_problem`` / ``load_problem``): the exact ``ba_problem``
  arrays of ``include/ba_hip.h``, little-endian, no pickling.  Lossless, so a
  problem gathered by ``prepareConstraints`` (Optimizer.cpp:279-333) on one
  host can be solved with Ceres on another and compared bit-for-bit on the
  inputs.  ``bundleadjustment_amd/host/ba_io.hpp`` reads and writes the same
  bytes from C++ (the side a Ceres-equipped host would compile).

  Layout: 8-byte magic ``b"BASOA\\0\\0\\1"``; int32 n_cams, n_pts, n_obs,
  flags (bit 0: cam_fixed + cam_fixed_extr present, bit 1: pt_fixed
  present); float64 huber_a; then cams f64[6C], K f32[9C],
  [cam_fixed u8[C], cam_fixed_extr f32[16C]], pts f64[3P], [pt_fixed u8[P]],
  obs_cam i32[N], obs_pt i32[N], obs_uv f32[2N].

* **BAL** (Bundle Adjustment in the Large, text): ``<C> <P> <N>``, N lines
  ``cam pt u v``, then 9 values per camera (angle-axis 3, t 3, f, k1, k2) and
  3 per point.  BAL projects p = -(R X + t) / (R X + t)_z, uv = f r(p) p with
  r(p) = 1 + k1 |p|^2 + k2 |p|^4.  The reference's functor has no distortion
  (r = hnormalized(K (R X + t)) - uv), so an undistorted BAL camera maps
  exactly to the same angle-axis and translation with K = diag(-f, -f, 1):
  q0 / q2 = -f P_x / P_z.  Cameras with k1 or k2 != 0 have no exact image in
  this model: ``distortion="reject"`` (default) refuses them,
  ``"ignore"`` drops the coefficients, and ``"undistort"`` maps each
  observation to the undistorted p (fixed-point solve of p' = r(p) p), an
  approximation of the BAL cost, not BAL's exact residual.
"""
from __future__ import annotations

import bz2
import gzip
import io
import os
import struct

import numpy as np

from .problem import HUBER_A, Problem

BAS_MAGIC = b"BASOA\0\0\1"
_FLAG_CAM_FIXED = 1
_FLAG_PT_FIXED = 2


# ---------------------------------------------------------------------------
# binary SoA dump
# ---------------------------------------------------------------------------
def save_problem(path: str | os.PathLike, problem: Problem) -> None:
    """Write the C-ABI arrays of ``problem`` (lossless)."""
    p = problem.normalized()
    flags = 0
    if p.cam_fixed is not None:
        flags |= _FLAG_CAM_FIXED
    if p.pt_fixed is not None:
        flags |= _FLAG_PT_FIXED
    with open(path, "wb") as f:
        f.write(BAS_MAGIC)
        f.write(struct.pack("<4i", p.n_cams, p.n_pts, p.n_obs, flags))
        f.write(struct.pack("<d", float(p.huber_a)))
        f.write(p.cams.astype("<f8").tobytes())
        f.write(p.K.astype("<f4").tobytes())
        if flags & _FLAG_CAM_FIXED:
            extr = p.cam_fixed_extr if p.cam_fixed_extr is not None else np.zeros((p.n_cams, 16), np.float32)
            f.write(p.cam_fixed.astype(np.uint8).tobytes())
            f.write(np.ascontiguousarray(extr, dtype="<f4").tobytes())
        f.write(p.pts.astype("<f8").tobytes())
        if flags & _FLAG_PT_FIXED:
            f.write(p.pt_fixed.astype(np.uint8).tobytes())
        f.write(p.obs_cam.astype("<i4").tobytes())
        f.write(p.obs_pt.astype("<i4").tobytes())
        f.write(p.obs_uv.astype("<f4").tobytes())


def load_problem(path: str | os.PathLike) -> Problem:
    """Read a BAS dump (validates sizes and indices; raises ValueError)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != BAS_MAGIC:
        raise ValueError(f"{path}: not a BAS problem dump")
    C, P, N, flags = struct.unpack_from("<4i", data, 8)
    (huber_a,) = struct.unpack_from("<d", data, 24)
    if min(C, P, N) < 0:
        raise ValueError(f"{path}: negative sizes")
    off = 32

    def take(dtype, count):
        nonlocal off
        nbytes = np.dtype(dtype).itemsize * count
        if off + nbytes > len(data):
            raise ValueError(f"{path}: truncated")
        a = np.frombuffer(data, dtype=dtype, count=count, offset=off).copy()
        off += nbytes
        return a

    cams = take("<f8", 6 * C).reshape(C, 6)
    K = take("<f4", 9 * C).reshape(C, 9)
    cam_fixed = extr = pt_fixed = None
    if flags & _FLAG_CAM_FIXED:
        cam_fixed = take(np.uint8, C)
        extr = take("<f4", 16 * C).reshape(C, 16)
    pts = take("<f8", 3 * P).reshape(P, 3)
    if flags & _FLAG_PT_FIXED:
        pt_fixed = take(np.uint8, P)
    obs_cam = take("<i4", N)
    obs_pt = take("<i4", N)
    uv = take("<f4", 2 * N).reshape(N, 2)
    if off != len(data):
        raise ValueError(f"{path}: {len(data) - off} trailing bytes")
    _check_indices(obs_cam, obs_pt, C, P, path)
    return Problem(cams=cams, K=K, pts=pts, obs_cam=obs_cam, obs_pt=obs_pt, obs_uv=uv, cam_fixed=cam_fixed,
                   cam_fixed_extr=extr, pt_fixed=pt_fixed, huber_a=huber_a,
                   name=os.path.basename(os.fspath(path))).normalized()


def _check_indices(obs_cam, obs_pt, C, P, where):
    if len(obs_cam) and (obs_cam.min() < 0 or obs_cam.max() >= C or obs_pt.min() < 0 or obs_pt.max() >= P):
        raise ValueError(f"{where}: observation index out of range")


# ---------------------------------------------------------------------------
# BAL text format
# ---------------------------------------------------------------------------
def _open_text(path):
    path = os.fspath(path)
    if path.endswith(".bz2"):
        return io.TextIOWrapper(bz2.open(path, "rb"))
    if path.endswith(".gz"):
        return io.TextIOWrapper(gzip.open(path, "rb"))
    return open(path, "r")


def _undistort(pd: np.ndarray, k1: np.ndarray, k2: np.ndarray, iters: int = 20) -> np.ndarray:
    """p with p' = (1 + k1 |p|^2 + k2 |p|^4) p (fixed-point, per row)."""
    p = pd.copy()
    for _ in range(iters):
        r2 = np.einsum("ij,ij->i", p, p)
        p = pd / (1.0 + k1 * r2 + k2 * r2 * r2)[:, None]
    return p


def read_bal(path: str | os.PathLike, distortion: str = "reject", huber_a: float = HUBER_A) -> Problem:
    """Read a BAL problem into the reference layout (see module docstring)."""
    if distortion not in ("reject", "ignore", "undistort"):
        raise ValueError("distortion must be 'reject', 'ignore' or 'undistort'")
    with _open_text(path) as f:
        head = f.readline().split()
        if len(head) != 3:
            raise ValueError(f"{path}: bad BAL header")
        C, P, N = (int(x) for x in head)
        vals = np.array(f.read().split(), dtype=np.float64)
    need = 4 * N + 9 * C + 3 * P
    if vals.size < need:
        raise ValueError(f"{path}: truncated ({vals.size} of {need} values)")
    obs = vals[:4 * N].reshape(N, 4)
    cam9 = vals[4 * N:4 * N + 9 * C].reshape(C, 9)
    pts = vals[4 * N + 9 * C:need].reshape(P, 3).copy()
    obs_cam = obs[:, 0].astype(np.int32)
    obs_pt = obs[:, 1].astype(np.int32)
    _check_indices(obs_cam, obs_pt, C, P, path)
    uv = obs[:, 2:4].copy()
    f, k1, k2 = cam9[:, 6], cam9[:, 7], cam9[:, 8]
    dist = (k1 != 0.0) | (k2 != 0.0)
    if np.any(dist):
        if distortion == "reject":
            raise ValueError(f"{path}: {int(dist.sum())} cameras have radial distortion (the reference model has "
                             "none); pass distortion='ignore' or 'undistort'")
        if distortion == "undistort":
            fo = f[obs_cam]
            pd = uv / fo[:, None]
            uv = _undistort(pd, k1[obs_cam], k2[obs_cam]) * fo[:, None]
    cams = np.ascontiguousarray(cam9[:, :6])
    K = np.zeros((C, 9), np.float32)
    K[:, 0] = -f          # column-major: K00
    K[:, 4] = -f          # K11
    K[:, 8] = 1.0         # K22
    return Problem(cams=cams, K=K, pts=pts, obs_cam=obs_cam, obs_pt=obs_pt, obs_uv=uv.astype(np.float32),
                   huber_a=huber_a, name=os.path.basename(os.fspath(path))).normalized()


def write_bal(path: str | os.PathLike, problem: Problem) -> None:
    """Write ``problem`` as BAL.  Requires K = [[fx, 0, cx], [0, fx, cy], [0, 0, 1]]
    per camera: BAL's f is -fx and the principal point is subtracted from the
    observations (the residuals are unchanged; reading back gives cx = cy = 0).
    Fixed-camera / fixed-point flags have no BAL encoding and are refused."""
    p = problem.normalized()
    if (p.cam_fixed is not None and p.cam_fixed.any()) or (p.pt_fixed is not None and p.pt_fixed.any()):
        raise ValueError("BAL has no constant parameter blocks; use save_problem for anchored problems")
    K = p.K.astype(np.float64).reshape(-1, 3, 3).transpose(0, 2, 1)   # row-major view
    fx, fy, cx, cy = K[:, 0, 0], K[:, 1, 1], K[:, 0, 2], K[:, 1, 2]
    if not (np.all(fx == fy) and np.all(K[:, 0, 1] == 0) and np.all(K[:, 1, 0] == 0) and np.all(K[:, 2, :2] == 0)
            and np.all(K[:, 2, 2] == 1)):
        raise ValueError("BAL needs fx == fy, zero skew and a last K row [0, 0, 1]")
    uv = p.obs_uv.astype(np.float64) - np.stack([cx[p.obs_cam], cy[p.obs_cam]], 1)
    with open(path, "w") as f:
        f.write(f"{p.n_cams} {p.n_pts} {p.n_obs}\n")
        for c, q, (u, v) in zip(p.obs_cam, p.obs_pt, uv):
            f.write(f"{int(c)} {int(q)} {float(u)!r} {float(v)!r}\n")
        for c in range(p.n_cams):
            for x in p.cams[c]:
                f.write(f"{float(x)!r}\n")
            f.write(f"{float(-fx[c])!r}\n0.0\n0.0\n")
        for x in p.pts.reshape(-1):
            f.write(f"{float(x)!r}\n")
