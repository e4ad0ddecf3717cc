"""BASELINE.json configs C4 and C5 on the HIP path at their per-GPU shard
sizes, and the reference's gauge-free observable output against the oracle.

C4 (configs[3]) is 1k cams x 1M pts x 10M obs with the points sharded over 8
GPUs; C5 (configs[4]) is 10k x 10M x 100M over 8 GPUs with fp32
mixed-precision Schur.  A rank holds 1/8 of the points
with all their observations and every camera, so the per-GPU problems are
make_config("c4" | "c5", scale=0.125): the camera side (the reduced system,
the CG) is full size, the observation side is one shard.

Observable output (Optimizer.cpp:252-267, the float write-back) in the
reference's own setting — only keyframe 0 anchored (Optimizer.cpp:314-321),
so the scale is free: the GPU and the oracle outputs are compared after a
Sim(3) alignment, together with the gauge-invariant per-observation
residuals and the outlier bits of pruneCorrespondences (Optimizer.cpp:6-79)
evaluated on each output.

Tolerances (besides those of test_gpu_parity.py):
  C4 shard vs oracle, 3 LM iterations ... cost rtol 1e-10, identical
      accept/reject decisions and CG iteration counts, parameters 1e-8
  C5 shard (MIXED_FP32) ................. properties: finite, accepted costs
      monotone, bitwise deterministic, final cost within 1e-6 of the fp64
      path
  10k-camera ITERATIVE_SCHUR vs oracle .. cost rtol 1e-9 and identical CG
      counts, fp64 and MIXED_FP32 (the oracle's rank-2 fp32 restatement,
      precision 3)
  C5 shard at full size, MIXED_FP32 vs the oracle's precision 3, 2 LM
      iterations ...................... cost rtol 1e-9, identical decisions
      and CG counts
  converged gauge-free output (200 LM iterations, tight tolerances) ...
      cost 1e-9; after the Sim(3) aligning the camera centres: centres and
      points (99th percentile) 1e-5 of the scene extent (float resolution
      ~6e-8), rotations 1e-5; residuals 1e-4 px (99th percentile); outlier
      bits <= 1 in 10^4 (0 measured)
  the reference's options (stops at function_tolerance 1e-6) ... cost 1e-6,
      aligned outputs 1e-3, residuals 1e-2 px, outlier bits <= 1 in 10^4
"""
import numpy as np
import pytest

from bundleadjustment_amd import Options, Solver, make_config, make_synthetic
from bundleadjustment_amd import problem as bp
from conftest import assert_close, compare_logs

from writeback import assert_float_output_within_1ulp  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver():
    s = Solver(0)
    yield s
    s.close()


def run_gpu(solver, p, opts):
    solver.set_problem(p)
    summ = solver.solve(opts)
    cams, pts = solver.params()
    return cams, pts, summ, solver.iteration_log()


def cg_counts(log):
    return [r["linear_solver_iterations"] for r in log[1:]]


# ---------------------------------------------------------------------------
# C4: one rank's shard of the 1k x 1M x 10M problem
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c4_shard():
    return make_config("c4", scale=0.125)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("lin", ["DENSE_SCHUR", "ITERATIVE_SCHUR"])
def test_c4_shard_first_iterations_match_oracle(solver, oracle_lib, c4_shard, lin):
    """1000 cameras (a 5994-row reduced system: 94 Cholesky block steps on
    the split path) x 125k points x 1.25M observations."""
    p = c4_shard
    assert p.n_cams == 1000 and p.n_obs > 1_000_000
    it = lin == "ITERATIVE_SCHUR"
    opts = Options(max_num_iterations=3, linear_solver_type=lin,
                   preconditioner_type="SCHUR_JACOBI" if it else "JACOBI")
    cams, pts, summ, glog = run_gpu(solver, p, opts)
    oc, op, osum, olog = oracle_lib.solve(p, oracle_lib.default_options(
        max_num_iterations=3, linear_solver=int(it), preconditioner_type=int(it)))
    compare_logs(glog, olog, rtol_cost=1e-10)
    assert cg_counts(glog) == cg_counts(olog)
    assert summ.final_cost < summ.initial_cost
    assert_close(cams, oc, 1e-8, 1e-10, "cameras")
    assert_close(pts, op, 1e-8, 1e-10, "points")
    assert_float_output_within_1ulp(cams, pts, oc, op, f"C4 shard {lin}")   # SURVEY.md §8c float-cast bar


# ---------------------------------------------------------------------------
# C5: one rank's shard of the 10k x 10M x 100M problem (12.5M observations),
# ITERATIVE_SCHUR with the W blocks stored in fp32
# ---------------------------------------------------------------------------
@pytest.mark.timeout(900)
def test_c5_shard_mixed_precision_properties():
    p = make_config("c5", scale=0.125)
    assert p.n_cams == 10_000 and p.n_obs > 12_000_000
    kw = dict(linear_solver_type="ITERATIVE_SCHUR", preconditioner_type="SCHUR_JACOBI", max_num_iterations=8)
    with Solver(0) as s:
        s.set_problem(p)
        sm = s.solve(Options(precision="MIXED_FP32", **kw))
        log_m = s.iteration_log()
        cm, xm = s.params()
        # bitwise deterministic
        s.set_params(p.cams, p.pts)
        sm2 = s.solve(Options(precision="MIXED_FP32", **kw))
        cm2, xm2 = s.params()
        # the fp64 path on the same shard (per-observation product matvec:
        # the fp64 W outgrows the Infinity Cache at this size)
        s.set_params(p.cams, p.pts)
        sd = s.solve(Options(**kw))
        log_d = s.iteration_log()
    assert sm.termination_type != "FAILURE" and sd.termination_type != "FAILURE"
    assert np.isfinite(cm).all() and np.isfinite(xm).all()
    accepted = [r["cost"] for r in log_m if r["step_is_successful"]]
    assert all(b <= a for a, b in zip(accepted, accepted[1:])), accepted
    assert sm.final_cost < 0.9 * sm.initial_cost   # (5 % gross outliers keep a large Huber cost)
    assert all(r["linear_solver_iterations"] >= 1 for r in log_m[1:])
    assert sm2.final_cost == sm.final_cost and np.array_equal(cm, cm2) and np.array_equal(xm, xm2)
    assert sm.final_cost == pytest.approx(sd.final_cost, rel=1e-6)
    for a, b in list(zip(log_m, log_d))[:4]:
        assert a["cost"] == pytest.approx(b["cost"], rel=1e-6)


@pytest.mark.timeout(900)
def test_c5_shard_mixed_precision_matches_oracle(solver, oracle_lib):
    """The full-size C5 shard (10k cameras x 1.25M points x 12.5M
    observations) in its own precision mode: MIXED_FP32 (the rank-2 records
    c, Z in fp32, the back substitution from the CG's accumulated products)
    against the oracle's restatement of those fp32 records (precision 3),
    2 LM iterations: costs 1e-9, identical accept/reject decisions and CG
    counts (Optimizer.cpp:242)."""
    p = make_config("c5", scale=0.125)
    assert p.n_cams == 10_000 and p.n_obs > 12_000_000
    opts = Options(max_num_iterations=2, linear_solver_type="ITERATIVE_SCHUR", preconditioner_type="SCHUR_JACOBI",
                   precision="MIXED_FP32")
    cams, pts, summ, glog = run_gpu(solver, p, opts)
    oc, op, osum, olog = oracle_lib.solve(p, oracle_lib.default_options(
        max_num_iterations=2, linear_solver=1, preconditioner_type=1, precision=3))
    compare_logs(glog, olog, rtol_cost=1e-9)
    assert cg_counts(glog) == cg_counts(olog)
    assert [r["step_is_successful"] for r in glog] == [r["step_is_successful"] for r in olog]
    assert summ.final_cost == pytest.approx(osum["final_cost"], rel=1e-9)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("precision", ["FP64", "MIXED_FP32"])
def test_10k_cameras_iterative_matches_oracle(solver, oracle_lib, precision):
    """C5's camera count (10k cameras, 60k camera unknowns: the grid-kernel CG)
    on a reduced point set, against the oracle's ITERATIVE_SCHUR — in fp64,
    and with the rank-2 W records (c, Z) rounded to fp32 (the oracle's
    independent restatement of MIXED_FP32 on those records, precision 3 of
    oracle/ba_oracle.cpp iterative_schur_solve_w)."""
    p = make_synthetic(10_000, 60_000, 10, seed=0xBA5E0004)
    assert p.n_cams == 10_000
    opts = Options(max_num_iterations=4, linear_solver_type="ITERATIVE_SCHUR", preconditioner_type="SCHUR_JACOBI",
                   precision=precision)
    cams, pts, summ, glog = run_gpu(solver, p, opts)
    # MIXED_FP32 beyond 200 cameras runs the point pass over the 16-value
    # rank-2 records with c and Z rounded to float (k_obs_w_rc<float, .., PC>):
    # the oracle's precision 3, not precision 1 (which rounds the 18 W entries)
    oc, op, osum, olog = oracle_lib.solve(p, oracle_lib.default_options(
        max_num_iterations=4, linear_solver=1, preconditioner_type=1, precision=3 if precision == "MIXED_FP32" else 0))
    compare_logs(glog, olog, rtol_cost=1e-9)
    assert cg_counts(glog) == cg_counts(olog)
    assert summ.final_cost == pytest.approx(osum["final_cost"], rel=1e-9)


# ---------------------------------------------------------------------------
# observable output at the reference's gauge (single anchor)
# ---------------------------------------------------------------------------
def write_back(cams, pts):
    """Optimizer.cpp:252-267: the float extrinsic [R(w) | t] (Matrix3d cast to
    float, t cast to float; the frame stores its inverse) and the float point."""
    R = bp.angle_axis_to_rotation(cams[:, :3]).astype(np.float32)
    t = cams[:, 3:].astype(np.float32)
    return R, t, pts.astype(np.float32)


def sim3_align(src, dst):
    """Umeyama: s, R, t minimising |s R src + t - dst|^2 (rows are points)."""
    ms, md = src.mean(0), dst.mean(0)
    a, b = src - ms, dst - md
    U, S, Vt = np.linalg.svd(b.T @ a / len(src))
    D = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        D[2, 2] = -1
    R = U @ D @ Vt
    s = np.trace(np.diag(S) @ D) / (a ** 2).sum(1).mean()
    return s, R, md - s * R @ ms


def outlier_bits(oracle_lib, p, R, t, X):
    """pruneCorrespondences on a written-back state: octave 0, no depth limits
    (the synthetic problem has neither), so the behind-camera and reprojection
    tests decide."""
    nc = p.n_cams
    extr = np.zeros((nc, 16), np.float32)
    for c in range(nc):
        E = np.eye(4, dtype=np.float32)
        E[:3, :3], E[:3, 3] = R[c], t[c]
        extr[c] = E.flatten(order="F")
    center = np.einsum("cji,cj->ci", R.astype(np.float64), -t.astype(np.float64)).astype(np.float32)
    n = p.n_obs
    return oracle_lib.prune(extr, center, p.K, p.obs_cam, X[p.obs_pt], p.obs_uv, np.ones(n, np.float32),
                            np.tile(np.array([0.0, 1e30], np.float32), (n, 1)))


def output_deviation(oracle_lib, solver, p, gpu, ora):
    """Written-back outputs of two solutions: the Sim(3) aligning the camera
    centres (GPU -> oracle), the aligned camera-centre, rotation and point
    deviations (relative to the scene extent), the per-observation residual
    difference and the two outlier-bit vectors."""
    (cams, pts), (oc, op) = gpu, ora
    Rg, tg, Xg = write_back(cams, pts)
    Ro, to, Xo = write_back(oc, op)
    cg = np.einsum("cji,cj->ci", Rg.astype(np.float64), -tg.astype(np.float64))
    co = np.einsum("cji,cj->ci", Ro.astype(np.float64), -to.astype(np.float64))
    s, Ra, ta = sim3_align(cg, co)
    extent = np.abs(co - co.mean(0)).max()
    dcam = np.abs((s * (Ra @ cg.T)).T + ta - co).max() / extent
    Xa = (s * (Ra @ Xg.astype(np.float64).T)).T + ta
    dpt = np.linalg.norm(Xa - Xo, axis=1) / extent
    rot = max(np.abs(Ra @ Rg[c].astype(np.float64).T - Ro[c].astype(np.float64).T).max() for c in range(p.n_cams))
    solver.set_params(cams, pts)
    rg, _ = solver.residuals()
    q = p.copy()
    q.cams, q.pts = oc, op
    ro = oracle_lib.residuals(q)
    bg = outlier_bits(oracle_lib, p, Rg, tg, Xg)
    bo = outlier_bits(oracle_lib, p, Ro, to, Xo)
    return dict(scale=s, cam=dcam, rot=rot, pt=dpt, resid=np.abs(rg - ro).max(), resid_all=np.abs(rg - ro).max(1),
                bits=(bg, bo))


@pytest.mark.timeout(600)
def test_gauge_free_converged_output_matches_oracle(solver, oracle_lib):
    """c2 (50 keyframes, Replica intrinsics), keyframe 0 the only anchor.  Run
    to tight tolerances (200 LM iterations) so both solvers sit at the
    minimum; the free scale drifts differently in each (rounding along the
    null space), so the written-back float poses and points are compared after
    the Sim(3) that aligns the camera centres, and the gauge-invariant
    quantities (costs, per-observation residuals, outlier bits) directly."""
    p = make_config("c2")
    kw = dict(max_num_iterations=200, function_tolerance=1e-13, gradient_tolerance=1e-16, parameter_tolerance=1e-14)
    cams, pts, summ, glog = run_gpu(solver, p, Options(**kw))
    # one oracle thread: its OpenMP reduction order would otherwise move the
    # trajectory along the free gauge from run to run
    oracle_lib.set_threads(1)
    try:
        oc, op, osum, olog = oracle_lib.solve(p, oracle_lib.default_options(**kw))
    finally:
        oracle_lib.set_threads(oracle_lib.max_threads())
    assert summ.termination_type != "FAILURE" and osum["termination_type"] != "FAILURE"
    compare_logs(glog, olog, n=10)
    assert summ.final_cost == pytest.approx(osum["final_cost"], rel=1e-9)
    d = output_deviation(oracle_lib, solver, p, (cams, pts), (oc, op))
    dcam, rot_dev, dpt = d["cam"], d["rot"], d["pt"]
    bg, bo = d["bits"]
    rr = d["resid_all"]
    stats = dict(scale=d["scale"], cam=dcam, rot=rot_dev, pt99=np.percentile(dpt, 99), ptmax=dpt.max(),
                 r99=np.percentile(rr, 99), rmax=rr.max(), bits=int((bg != bo).sum()), outliers=int((bg != 0).sum()))
    # measured (MI355X, this seed, four runs): scale 1 + O(1e-3) (the free
    # gauge), camera centres 0.3-1.8e-7, rotations 0.04-1.7e-7, points p99
    # 2.6-3.5e-8 of the extent (float resolution ~6e-8), 0 of 2683 outlier
    # bits differ.  Maxima over points / residuals are set by the few
    # near-degenerate triangulations (small baseline, or observed mostly
    # through the linear Huber branch: the cost is nearly flat along them)
    # and vary run to run (points 6e-8 .. 4.5e-4 of the extent, residuals
    # 1.8e-5 .. 0.24 px); the bulk statistics are what is pinned.
    ok = (stats["cam"] < 1e-5 and stats["rot"] < 1e-5 and stats["pt99"] < 1e-5 and stats["ptmax"] < 1e-2
          and stats["r99"] < 1e-4 and stats["rmax"] < 1.0 and stats["bits"] <= max(1, p.n_obs // 10_000)
          and 0 < stats["outliers"] < p.n_obs)
    assert ok, stats


@pytest.mark.timeout(600)
def test_gauge_free_reference_options_output(solver, oracle_lib):
    """The reference's own options (Ceres defaults, 50 iterations): the two
    solvers stop within the function tolerance of the same minimum; outputs
    agree to the precision that stopping rule leaves."""
    p = make_config("c2")
    cams, pts, summ, glog = run_gpu(solver, p, Options(max_num_iterations=50))
    oc, op, osum, olog = oracle_lib.solve(p, oracle_lib.default_options(max_num_iterations=50))
    compare_logs(glog, olog, n=10)
    assert summ.final_cost == pytest.approx(osum["final_cost"], rel=1e-6)
    d = output_deviation(oracle_lib, solver, p, (cams, pts), (oc, op))
    assert d["cam"] < 1e-3 and d["rot"] < 1e-4 and np.percentile(d["pt"], 99) < 1e-3, d
    assert d["resid"] < 1e-2, d["resid"]
    bg, bo = d["bits"]
    assert (bg != bo).sum() <= max(1, p.n_obs // 10_000)
