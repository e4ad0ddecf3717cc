"""Batched pose-only solves: ba_solve_pose_batch runs
MotionOnlyBAOptimizerAngles' Ceres solve (Optimizer.cpp:417-442,
PoseOnlyAngleReprojectionError Optimizer.h:163-182 + HuberLoss) for many
frames in one launch.  Each problem is checked against the oracle's LM on
the equivalent one-camera problem (same tolerances as test_gpu_parity:
final cost 1e-10 rel, camera 1e-8 rel + 1e-10 abs, identical termination,
iteration and successful-step counts) and against ba_solve on the device."""
import numpy as np
import pytest

from bundleadjustment_amd import Options, Solver, make_synthetic
from bundleadjustment_amd import problem as bp
from bundleadjustment_amd._native import BAError
from conftest import assert_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver():
    s = Solver(0)
    yield s
    s.close()


def f2f_problem(n_obs, seed, intr="freiburg", huber=True, noise_px=1.0, outlier_frac=0.05):
    """One frame: one variable camera, constant points (make_synthetic's
    motion-only mode: points rounded through float like Vector4f)."""
    p = make_synthetic(1, max(n_obs, 1), 1, seed=seed, intr=intr, motion_only=True, noise_px=noise_px,
                       outlier_frac=outlier_frac)
    if n_obs == 0:
        p.obs_cam = p.obs_cam[:0]
        p.obs_pt = p.obs_pt[:0]
        p.obs_uv = p.obs_uv[:0]
    if not huber:
        p.huber_a = 0.0
    return p.normalized()


def batch_of(problems):
    off = np.zeros(len(problems) + 1, np.int32)
    cams, K, X, uv = [], [], [], []
    for i, p in enumerate(problems):
        off[i + 1] = off[i] + p.n_obs
        cams.append(p.cams[0])
        K.append(p.K[0])
        X.append(p.pts[p.obs_pt])
        uv.append(p.obs_uv)
    return off, np.array(cams), np.array(K), np.concatenate(X), np.concatenate(uv)


def check_against_oracle(oracle_lib, p, cam, summ, opts):
    oc, _, osum, _ = oracle_lib.solve(p, opts)
    assert summ.termination_type == osum["termination_type"], (summ, osum)
    assert summ.num_iterations == osum["num_iterations"], (summ, osum)
    assert summ.num_successful_steps == osum["num_successful_steps"], (summ, osum)
    assert summ.initial_cost == pytest.approx(osum["initial_cost"], rel=1e-12)
    assert summ.final_cost == pytest.approx(osum["final_cost"], rel=1e-10)
    assert_close(cam, oc[0], 1e-8, 1e-10, "camera")


@pytest.mark.parametrize("n_obs", [300, 2000])
def test_single_frame_matches_oracle_and_ba_solve(solver, oracle_lib, n_obs):
    p = f2f_problem(n_obs, seed=0xF2F0 + n_obs)
    off, cams, K, X, uv = batch_of([p])
    out, summs = solver.solve_pose_batch(off, cams, K, X, uv, Options(max_num_iterations=20))
    check_against_oracle(oracle_lib, p, out[0], summs[0], oracle_lib.default_options(max_num_iterations=20))
    solver.set_problem(p)
    s2 = solver.solve(Options(max_num_iterations=20))
    c2, _ = solver.params()
    assert s2.num_iterations == summs[0].num_iterations
    assert s2.final_cost == pytest.approx(summs[0].final_cost, rel=1e-10)
    assert_close(out[0], c2[0], 1e-8, 1e-10, "camera vs ba_solve")


def test_batch_of_mixed_sizes_matches_oracle(solver, oracle_lib):
    """64 frames of ragged sizes (1 .. 1500 observations, both intrinsics)."""
    rng = np.random.default_rng(21)
    sizes = [1, 2, 5, 63, 64, 65, 128, 1500] + list(rng.integers(10, 800, 56))
    probs = [f2f_problem(int(n), seed=1000 + i, intr="replica" if i % 3 == 0 else "freiburg")
             for i, n in enumerate(sizes)]
    off, cams, K, X, uv = batch_of(probs)
    opts = Options(max_num_iterations=20)
    out, summs = solver.solve_pose_batch(off, cams, K, X, uv, opts)
    for i, p in enumerate(probs):
        check_against_oracle(oracle_lib, p, out[i], summs[i], oracle_lib.default_options(max_num_iterations=20))


def test_no_loss_no_scaling_and_iteration_cap(solver, oracle_lib):
    probs = [f2f_problem(400, seed=77, huber=False), f2f_problem(250, seed=78)]
    off, cams, K, X, uv = batch_of(probs)
    out, summs = solver.solve_pose_batch(off, cams, K, X, uv, Options(max_num_iterations=3, jacobi_scaling=False),
                                         huber_a=0.0)
    check_against_oracle(oracle_lib, probs[0], out[0], summs[0],
                         oracle_lib.default_options(max_num_iterations=3, jacobi_scaling=0))
    # huber_a is per batch: problem 1 also solved without loss
    p1 = probs[1].copy()
    p1.huber_a = 0.0
    check_against_oracle(oracle_lib, p1, out[1], summs[1],
                         oracle_lib.default_options(max_num_iterations=3, jacobi_scaling=0))


def test_noise_free_recovers_pose(solver):
    probs = [f2f_problem(500, seed=300 + i, noise_px=0.0, outlier_frac=0.0) for i in range(8)]
    off, cams, K, X, uv = batch_of(probs)
    out, summs = solver.solve_pose_batch(off, cams, K, X, uv)
    for p, c, s in zip(probs, out, summs):
        assert s.termination_type == "CONVERGENCE"
        assert np.allclose(c, p.gt_cams[0], atol=2e-5), (c, p.gt_cams[0])   # float-rounded points


def test_empty_frames_and_errors(solver):
    probs = [f2f_problem(0, seed=5), f2f_problem(100, seed=6), f2f_problem(0, seed=7)]
    off, cams, K, X, uv = batch_of(probs)
    out, summs = solver.solve_pose_batch(off, cams, K, X, uv)
    assert np.array_equal(out[0], cams[0]) and np.array_equal(out[2], cams[2])
    assert summs[0].termination_type == "CONVERGENCE" and summs[0].num_iterations == 0
    assert summs[1].num_iterations > 0
    bad = off.copy()
    bad[2] = bad[1] - 1
    with pytest.raises(BAError, match="decreases"):
        solver.solve_pose_batch(bad, cams, K, X, uv)


def test_batch_is_deterministic(solver):
    probs = [f2f_problem(700, seed=900 + i) for i in range(16)]
    off, cams, K, X, uv = batch_of(probs)
    a, _ = solver.solve_pose_batch(off, cams, K, X, uv)
    b, _ = solver.solve_pose_batch(off, cams, K, X, uv)
    assert np.array_equal(a, b)
