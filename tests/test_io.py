"""Problem I/O: BAS dump round trips (Python and the
C++ header bundleadjustment_amd/host/ba_io.hpp, byte for byte), and the BAL
mapping checked against BAL's own projection formula.  CPU only."""
import math
import shutil
import subprocess

import numpy as np
import pytest

from bundleadjustment_amd import io as bio
from bundleadjustment_amd import problem as bp
from conftest import ROOT


def _same_problem(a, b):
    for f in ("cams", "K", "pts", "obs_cam", "obs_pt", "obs_uv", "cam_fixed", "cam_fixed_extr", "pt_fixed"):
        x, y = getattr(a, f), getattr(b, f)
        if x is None or y is None:
            assert x is None and y is None, f
            continue
        assert x.dtype == y.dtype and x.shape == y.shape, f
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), f   # bitwise (NaN-safe)
    assert a.huber_a == b.huber_a


@pytest.mark.parametrize("name", ["c1", "c2", "f2f"])
def test_bas_roundtrip(tmp_path, name):
    p = bp.make_config(name, scale=0.05 if name == "c2" else 1.0)
    path = tmp_path / "p.bas"
    bio.save_problem(path, p)
    _same_problem(bio.load_problem(path), p)


def test_bas_rejects_corrupt(tmp_path):
    p = bp.make_config("c1")
    path = tmp_path / "p.bas"
    bio.save_problem(path, p)
    data = path.read_bytes()
    (tmp_path / "trunc.bas").write_bytes(data[:-3])
    with pytest.raises(ValueError, match="truncated"):
        bio.load_problem(tmp_path / "trunc.bas")
    (tmp_path / "magic.bas").write_bytes(b"X" + data[1:])
    with pytest.raises(ValueError, match="not a BAS"):
        bio.load_problem(tmp_path / "magic.bas")
    bad = bytearray(data)
    off = len(data) - 8 * p.n_obs - 4 * p.n_obs - 4 * p.n_obs   # first obs_cam entry
    bad[off:off + 4] = np.int32(p.n_cams).tobytes()
    (tmp_path / "idx.bas").write_bytes(bytes(bad))
    with pytest.raises(ValueError, match="out of range"):
        bio.load_problem(tmp_path / "idx.bas")


def _bal_project(cam9, X):
    """BAL's published camera model: P = R X + t, p = -P / P_z, uv = f r(p) p."""
    R = bp.angle_axis_to_rotation(cam9[:, :3])
    P = np.einsum("nij,nj->ni", R, X) + cam9[:, 3:6]
    p = -P[:, :2] / P[:, 2:3]
    r2 = np.sum(p * p, 1)
    return cam9[:, 6:7] * (1.0 + cam9[:, 7] * r2 + cam9[:, 8] * r2 * r2)[:, None] * p


def _write_bal_text(path, cam9, pts, obs_cam, obs_pt, uv):
    with open(path, "w") as f:
        f.write(f"{len(cam9)} {len(pts)} {len(obs_cam)}\n")
        for c, q, (u, v) in zip(obs_cam, obs_pt, uv):
            f.write(f"{c} {q} {u:.17g} {v:.17g}\n")
        for x in cam9.reshape(-1):
            f.write(f"{x:.17g}\n")
        for x in pts.reshape(-1):
            f.write(f"{x:.17g}\n")


def _bal_scene(rng, n_cams=4, n_pts=30, k1=0.0, k2=0.0):
    cam9 = np.zeros((n_cams, 9))
    cam9[:, :3] = rng.normal(0, 0.2, (n_cams, 3))
    cam9[:, 3:5] = rng.normal(0, 0.3, (n_cams, 2))
    cam9[:, 5] = -6.0                     # BAL cameras look down -z
    cam9[:, 6] = rng.uniform(400, 600, n_cams)
    cam9[:, 7], cam9[:, 8] = k1, k2
    pts = rng.uniform(-1, 1, (n_pts, 3))
    obs_cam = np.repeat(np.arange(n_cams), n_pts).astype(np.int32)
    obs_pt = np.tile(np.arange(n_pts), n_cams).astype(np.int32)
    uv = _bal_project(cam9[obs_cam], pts[obs_pt])
    return cam9, pts, obs_cam, obs_pt, uv


def _model_residual(p):
    """The reference functor r = hnormalized(K (R X + t)) - uv (Optimizer.h:64-74)."""
    R = bp.angle_axis_to_rotation(p.cams[p.obs_cam, :3])
    proj, _ = bp.project(R, p.cams[p.obs_cam, 3:], p.K[p.obs_cam], p.pts[p.obs_pt])
    return proj - p.obs_uv.astype(np.float64)


def test_bal_read_matches_bal_projection(tmp_path):
    rng = np.random.default_rng(5)
    cam9, pts, oc, op, uv = _bal_scene(rng)
    _write_bal_text(tmp_path / "s.txt", cam9, pts, oc, op, uv)
    p = bio.read_bal(tmp_path / "s.txt")
    assert (p.n_cams, p.n_pts, p.n_obs) == (4, 30, 120)
    assert np.array_equal(p.cams, cam9[:, :6]) and np.array_equal(p.pts, pts)
    # residual = float32 rounding of the observations and of K only
    r = _model_residual(p)
    assert np.max(np.abs(r)) < 1e-3, np.max(np.abs(r))


def test_bal_distortion_modes(tmp_path):
    rng = np.random.default_rng(6)
    cam9, pts, oc, op, uv = _bal_scene(rng, k1=-0.05, k2=0.01)
    _write_bal_text(tmp_path / "d.txt", cam9, pts, oc, op, uv)
    with pytest.raises(ValueError, match="distortion"):
        bio.read_bal(tmp_path / "d.txt")
    pi = bio.read_bal(tmp_path / "d.txt", distortion="ignore")
    pu = bio.read_bal(tmp_path / "d.txt", distortion="undistort")
    assert np.max(np.abs(_model_residual(pu))) < 1e-3
    assert np.max(np.abs(_model_residual(pi))) > 0.1    # the dropped distortion shows


def test_bal_write_read_roundtrip(tmp_path):
    p = bp.make_config("c2", scale=0.02)
    p.cam_fixed = None
    p.cam_fixed_extr = None
    p.K[:, 6:8] = 0.0                     # BAL has no principal point
    path = tmp_path / "w.txt"
    bio.write_bal(path, p)
    q = bio.read_bal(path)
    assert np.array_equal(q.cams, p.cams) and np.array_equal(q.pts, p.pts)
    assert np.array_equal(q.obs_cam, p.obs_cam) and np.array_equal(q.obs_pt, p.obs_pt)
    assert np.array_equal(q.obs_uv, p.obs_uv)
    assert np.array_equal(np.abs(q.K), np.abs(p.K))   # f sign: BAL's -z convention
    assert np.allclose(_model_residual(q), _model_residual(p), atol=1e-9)


def test_bal_write_principal_point_shift(tmp_path):
    """K with (cx, cy): observations shifted, residuals unchanged."""
    p = bp.make_config("c1")
    p.cam_fixed = None
    p.cam_fixed_extr = None
    bio.write_bal(tmp_path / "c.txt", p)
    q = bio.read_bal(tmp_path / "c.txt")
    assert np.allclose(_model_residual(q), _model_residual(p), atol=1e-3)
    with pytest.raises(ValueError, match="constant"):
        bio.write_bal(tmp_path / "x.txt", bp.make_config("c1"))




@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_cpp_header_is_byte_compatible(tmp_path):
    src = ROOT / "tests" / "cpp" / "io_rt.cpp"      # also built with ASan + UBSan (tests/test_sanitize.py)
    exe = tmp_path / "io_rt"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", f"-I{ROOT / 'include'}",
                    f"-I{ROOT / 'bundleadjustment_amd' / 'host'}", str(src), "-o", str(exe)], check=True)
    p = bp.fix_camera(bp.make_config("c2", scale=0.02), 1)
    bio.save_problem(tmp_path / "a.bas", p)
    rng = np.random.default_rng(7)
    cam9, pts, oc, op, uv = _bal_scene(rng)
    _write_bal_text(tmp_path / "s.txt", cam9, pts, oc, op, uv)
    out = subprocess.run([str(exe), str(tmp_path / "a.bas"), str(tmp_path / "b.bas"), str(tmp_path / "s.txt"),
                          str(tmp_path / "s.bas")], check=True, capture_output=True, text=True).stdout
    assert out.split() == [str(p.n_cams), str(p.n_pts), str(p.n_obs)]
    assert (tmp_path / "a.bas").read_bytes() == (tmp_path / "b.bas").read_bytes()
    # the C++ BAL reader and the Python one agree bit for bit
    py = bio.read_bal(tmp_path / "s.txt", huber_a=2.0)
    _same_problem(bio.load_problem(tmp_path / "s.bas"), py)
