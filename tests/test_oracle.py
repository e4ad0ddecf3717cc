"""CPU tests of the oracle (the CPU restatement of the reference's Ceres path):
pinned against the golden functor vectors, rotation known-answer tests, and
LM known-answer tests.  No GPU."""
import math

import numpy as np
import pytest

from bundleadjustment_amd import problem as bp
from conftest import assert_close
from golden_problems import golden_expected, golden_problem


@pytest.mark.parametrize("kind", ["angle", "pose", "point"])
def test_oracle_matches_golden_functors(oracle_lib, golden, kind):
    """Oracle Jet autodiff == independent torch jacfwd restatement (Optimizer.h:54-76, 96-107, 163-182)."""
    p = golden_problem(golden, kind)
    r, J, cost, ok = oracle_lib.linearize(p)
    assert ok
    r_ref, J_ref = golden_expected(golden, kind)
    assert_close(r, r_ref, 1e-12, 1e-9, f"{kind} residual")
    assert_close(J, J_ref, 1e-11, 1e-9, f"{kind} jacobian")
    assert cost == pytest.approx(0.5 * np.sum(r_ref ** 2), rel=1e-12)


def test_huber_corrector(oracle_lib, golden):
    """ceres::HuberLoss(a) + Corrector: rho = 2a|r| - a^2 beyond a, r and J scaled by sqrt(a/|r|)."""
    a = math.sqrt(5.991)
    p = golden_problem(golden, "angle", huber_a=a)
    r0, J0 = golden_expected(golden, "angle")
    # move every other observation next to its projection (inlier region)
    rng = np.random.default_rng(1)
    inl = np.arange(p.n_obs) % 2 == 0
    uv_new = p.obs_uv.astype(np.float64).copy()
    uv_new[inl] += r0[inl] - rng.uniform(-1.5, 1.5, size=(inl.sum(), 2))
    p.obs_uv = uv_new.astype(np.float32)
    r0 = r0 + golden["uv"].astype(np.float64) - p.obs_uv.astype(np.float64)
    r, J, cost, _ = oracle_lib.linearize(p)
    s = np.sum(r0 ** 2, axis=1)
    out = s > a * a
    sc = np.where(out, np.sqrt(np.maximum(a / np.sqrt(s), np.finfo(float).tiny)), 1.0)
    assert_close(r, r0 * sc[:, None], 1e-11, 1e-9, "corrected residual")
    assert_close(J, J0 * sc[:, None, None], 1e-11, 1e-9, "corrected jacobian")
    rho = np.where(out, 2 * a * np.sqrt(s) - a * a, s)
    assert cost == pytest.approx(0.5 * rho.sum(), rel=1e-12)
    assert out.any() and (~out).any()


def test_rotation_known_answers(oracle_lib):
    rng = np.random.default_rng(7)
    # identity, first-order branch, generic, near pi
    assert np.allclose(oracle_lib.angle_axis_to_R(np.zeros(3)), np.eye(3), atol=0)
    w = np.array([1e-9, -2e-9, 3e-9])
    R = oracle_lib.angle_axis_to_R(w)
    assert np.array_equal(R, np.array([[1, -w[2], w[1]], [w[2], 1, -w[0]], [-w[1], w[0], 1]]))
    for _ in range(200):
        w = rng.normal(0, 1.0, 3)
        th = np.linalg.norm(w)
        if th > 3.1:
            continue
        R = oracle_lib.angle_axis_to_R(w)
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-14)
        assert np.linalg.det(R) == pytest.approx(1.0, abs=1e-14)
        # Rodrigues: R v = v for v || w
        assert np.allclose(R @ w, w, atol=1e-14)
        w2 = oracle_lib.R_to_angle_axis(R)
        assert np.allclose(w2, w, atol=1e-12)
        # numpy restatement in the product (used for gather / synthetic data)
        assert np.allclose(bp.rotation_to_angle_axis(R), w2, atol=0, rtol=0)
        assert np.allclose(bp.angle_axis_to_rotation(w), R, atol=1e-15)
    # near pi: the (trace < 0) Shepperd branch
    ax = np.array([0.3, -0.5, 0.81]); ax /= np.linalg.norm(ax)
    for th in (math.pi - 1e-3, math.pi - 1e-7):
        R = oracle_lib.angle_axis_to_R(ax * th)
        w2 = oracle_lib.R_to_angle_axis(R)
        assert np.linalg.norm(w2) == pytest.approx(th, abs=1e-6)
        assert np.allclose(oracle_lib.angle_axis_to_R(w2), R, atol=1e-12)


def test_rotation_derivative_finite_difference(oracle_lib):
    rng = np.random.default_rng(3)
    for _ in range(20):
        w = rng.normal(0, 0.8, 3)
        R, dR = oracle_lib.angle_axis_to_R_jac(w)
        h = 1e-6
        for k in range(3):
            e = np.zeros(3); e[k] = h
            fd = (oracle_lib.angle_axis_to_R(w + e) - oracle_lib.angle_axis_to_R(w - e)) / (2 * h)
            assert np.allclose(dR[k], fd, atol=1e-8)


def test_noise_free_converges_to_ground_truth(oracle_lib):
    """Known answer: a noise-free problem converges to zero cost; the solution
    equals ground truth up to the free scale gauge about the anchored camera."""
    p = bp.make_synthetic(12, 3000, 4, seed=11, noise_px=0.0, outlier_frac=0.0)
    cams, pts, s, log = oracle_lib.solve(p)
    assert s["termination_type"] == "CONVERGENCE"
    assert s["final_cost"] < 1e-10 * s["initial_cost"]
    # camera 0 (anchor) centre c0; points are gt scaled about c0
    R0 = bp.angle_axis_to_rotation(p.gt_cams[0, :3]); c0 = -R0.T @ p.gt_cams[0, 3:]
    a = (p.gt_pts - c0).ravel(); b = (pts - c0).ravel()
    scale = a @ b / (a @ a)
    assert np.allclose(pts - c0, scale * (p.gt_pts - c0), atol=1e-5)
    # iteration-log invariants
    assert log[0]["iteration"] == 0 and log[0]["step_is_successful"] == 1
    costs = [r["cost"] for r in log if r["step_is_successful"]]
    assert all(c1 <= c0 for c0, c1 in zip(costs, costs[1:]))


def _np_residuals(x, p, nc_var, var_cams, npts):
    """Independent plain-numpy residual (no loss) for scipy."""
    cams = p.cams.copy()
    cams[var_cams] = x[:6 * nc_var].reshape(-1, 6)
    pts = x[6 * nc_var:].reshape(npts, 3)
    R = bp.angle_axis_to_rotation(cams[p.obs_cam, :3])
    P = np.einsum("nij,nj->ni", R, pts[p.obs_pt]) + cams[p.obs_cam, 3:]
    K = p.K[p.obs_cam].astype(np.float64).reshape(-1, 3, 3).transpose(0, 2, 1)
    q = np.einsum("nij,nj->ni", K, P)
    return (q[:, :2] / q[:, 2:3] - p.obs_uv.astype(np.float64)).ravel()


def test_minimum_matches_scipy_least_squares(oracle_lib):
    """The LM/DENSE_SCHUR minimum equals scipy's (no robust loss, gauge fixed
    by anchoring two cameras so the minimiser is unique)."""
    from scipy.optimize import least_squares
    from scipy.sparse import lil_matrix
    p = bp.make_synthetic(8, 400, 4, seed=5, noise_px=1.0, outlier_frac=0.0)
    p.huber_a = 0.0
    # anchor camera 1 too (the angle reprojection functor on fixed cams is not
    # used here: fixing via cam_fixed + its float extrinsic)
    R1 = bp.angle_axis_to_rotation(p.cams[1, :3])
    p.cam_fixed[1] = 1
    p.cam_fixed_extr[1] = bp.extr_colmajor(R1, p.cams[1, 3:])
    Rf = p.cam_fixed_extr[1].reshape(4, 4).T[:3, :3].astype(np.float64)
    p.cams[1, :3] = bp.rotation_to_angle_axis(Rf)
    p.cams[1, 3:] = p.cam_fixed_extr[1].reshape(4, 4).T[:3, 3]
    opts = oracle_lib.default_options(max_num_iterations=200, function_tolerance=1e-15,
                                      parameter_tolerance=1e-14, gradient_tolerance=1e-14)
    cams, pts, s, _ = oracle_lib.solve(p, opts)
    var = np.arange(2, p.n_cams)
    # scipy residual uses the float extrinsic of fixed cams exactly like PointOnly: here the
    # fixed cams' angle-axis reproduce those extrinsics to float precision; evaluate fixed
    # cams through their float extrinsic to match the problem definition
    def fun(x):
        r = _np_residuals(x, p, len(var), var, p.n_pts).reshape(-1, 2)
        for c in (0, 1):
            sel = p.obs_cam == c
            E = p.cam_fixed_extr[c].reshape(4, 4).T.astype(np.float64)
            X = x[6 * len(var):].reshape(-1, 3)[p.obs_pt[sel]]
            ph = X @ E[:3, :3].T + E[:3, 3]
            ph = ph / (X @ E[3, :3] + E[3, 3])[:, None]
            K = p.K[c].astype(np.float64).reshape(3, 3).T
            q = ph @ K.T
            r[sel] = q[:, :2] / q[:, 2:3] - p.obs_uv[sel]
        return r.ravel()
    x0 = np.concatenate([p.cams[var].ravel(), p.pts.ravel()])
    sp = lil_matrix((2 * p.n_obs, x0.size), dtype=int)
    for o in range(p.n_obs):
        c, q = p.obs_cam[o], p.obs_pt[o]
        rows = [2 * o, 2 * o + 1]
        if c >= 2:
            j = 6 * (c - 2)
            sp[rows[0], j:j + 6] = 1; sp[rows[1], j:j + 6] = 1
        j = 6 * len(var) + 3 * q
        sp[rows[0], j:j + 3] = 1; sp[rows[1], j:j + 3] = 1
    res = least_squares(fun, x0, jac_sparsity=sp, method="trf", x_scale="jac", ftol=1e-15, xtol=1e-15,
                        gtol=1e-15, max_nfev=200)
    cost_scipy = 0.5 * np.sum(res.fun ** 2)
    assert s["final_cost"] == pytest.approx(cost_scipy, rel=1e-8)
    x_or = np.concatenate([cams[var].ravel(), pts.ravel()])
    assert np.allclose(x_or, res.x, rtol=0, atol=1e-6)
