"""ITERATIVE_SCHUR (implicit Schur complement + preconditioned CG; SURVEY.md
§8a-a7 / §8e): the oracle's restatement of Ceres' IterativeSchurComplementSolver
/ ConjugateGradientsSolver against DENSE_SCHUR (CPU), and the HIP path
(ba_pcg.hip, through the C ABI) against the oracle (GPU).

The reference itself only uses DENSE_SCHUR (Optimizer.cpp:85); ITERATIVE_SCHUR
is the scalable solver the survey names for C5-sized camera counts, so its
parity anchor is (a) the oracle's CG restated from Ceres and (b) the minimum
DENSE_SCHUR reaches on the same problem.

Tolerances:
  GPU vs oracle, per LM iteration ... cost rtol 1e-9, identical accept/reject
                                      decisions and CG iteration counts (the CG
                                      termination test zeta < eta is a
                                      discrete decision on rounding-level
                                      different iterates; the seeds below are
                                      checked not to sit on its edge)
  final cost vs DENSE_SCHUR ......... rtol 1e-9 on gauge-fixed problems run
                                      to a tight function tolerance (inexact
                                      Newton steps reach the same minimum)
"""
import numpy as np
import pytest

from bundleadjustment_amd import Options, make_config, make_synthetic
from bundleadjustment_amd import problem as bp

PRECONDITIONERS = ["JACOBI", "SCHUR_JACOBI"]
PC = {"JACOBI": 0, "SCHUR_JACOBI": 1}


def oracle_opts(oracle_lib, pc, **kw):
    return oracle_lib.default_options(linear_solver=1, preconditioner_type=PC[pc], **kw)


def with_duplicate_observations(p, n_dup=40, seed=3):
    """Observe some points twice by the same camera (two keypoints matched to
    one map point): the Schur-Jacobi diagonal block then carries cross terms."""
    rng = np.random.default_rng(seed)
    q = p.copy()
    idx = rng.choice(q.n_obs, n_dup, replace=False)
    q.obs_cam = np.concatenate([q.obs_cam, q.obs_cam[idx]]).astype(np.int32)
    q.obs_pt = np.concatenate([q.obs_pt, q.obs_pt[idx]]).astype(np.int32)
    uv = q.obs_uv.reshape(-1, 2)
    q.obs_uv = np.concatenate([uv, uv[idx] + rng.normal(0, 2.0, (n_dup, 2)).astype(np.float32)]).astype(np.float32)
    return q.normalized()


# ---------------------------------------------------------------------------
# oracle (CPU)
# ---------------------------------------------------------------------------
def gauge_fixed(cfg, scale):
    """Well-posed variant (a second anchored camera removes the free scale of
    the reference's single-anchor setting), so both solvers converge to one
    isolated minimum."""
    return bp.fix_camera(make_config(cfg, scale=scale), 1)


@pytest.mark.parametrize("pc", PRECONDITIONERS)
@pytest.mark.parametrize("cfg,scale", [("c2", 0.2), ("c3", 0.01)])
def test_oracle_iterative_reaches_dense_minimum(oracle_lib, cfg, scale, pc):
    p = gauge_fixed(cfg, scale)
    kw = dict(max_num_iterations=100, function_tolerance=1e-12)
    _, _, sd, _ = oracle_lib.solve(p, oracle_lib.default_options(**kw))
    _, _, si, log = oracle_lib.solve(p, oracle_opts(oracle_lib, pc, **kw))
    assert si["termination_type"] != "FAILURE"
    assert si["final_cost"] == pytest.approx(sd["final_cost"], rel=1e-9)
    assert all(r["linear_solver_iterations"] >= 1 for r in log[1:])


def test_oracle_schur_jacobi_is_exact_for_one_camera(oracle_lib):
    """One variable camera: the Schur-Jacobi preconditioner is S^-1, so CG
    reaches the exact step in its first iteration and stops at the second
    (zeta = 0 < eta)."""
    p = make_config("c1")
    _, _, _, log = oracle_lib.solve(p, oracle_opts(oracle_lib, "SCHUR_JACOBI", max_num_iterations=5))
    assert [r["linear_solver_iterations"] for r in log[1:]] == [2] * (len(log) - 1)


def test_oracle_residual_reset_and_iteration_cap(oracle_lib):
    """A tight forcing sequence runs CG past the residual-reset period (10)
    and into max_linear_solver_iterations; the steps stay valid."""
    p = make_config("c2", scale=0.2)
    o = oracle_opts(oracle_lib, "JACOBI", max_num_iterations=4, eta=1e-14, max_linear_solver_iterations=23)
    _, _, s, log = oracle_lib.solve(p, o)
    its = [r["linear_solver_iterations"] for r in log[1:]]
    assert max(its) == 23 and all(r["step_is_valid"] for r in log[1:])
    assert s["final_cost"] < s["initial_cost"]


@pytest.mark.parametrize("pc", PRECONDITIONERS)
def test_oracle_w_form_and_mixed_precision(oracle_lib, pc):
    """precision 2 (oracle test hook): the per-observation W-block form of the
    implicit reduced system, the form MIXED_FP32 rounds, restates Ceres' F/E
    form — identical CG counts, costs to 1e-12.  precision 1 (MIXED_FP32, W
    rounded to fp32) and 3 (MIXED_FP32 with W = c'Z, c and Z rounded to fp32
    in the matvec): final cost within 1e-6 of fp64."""
    p = gauge_fixed("c2", 0.5)
    runs = {}
    for prec in (0, 2, 1, 3):
        _, _, s, log = oracle_lib.solve(p, oracle_opts(oracle_lib, pc, max_num_iterations=12, precision=prec))
        runs[prec] = (s, log)
    s0, l0 = runs[0]
    s2, l2 = runs[2]
    assert [r["linear_solver_iterations"] for r in l2] == [r["linear_solver_iterations"] for r in l0]
    for a, b in zip(l2, l0):
        assert a["cost"] == pytest.approx(b["cost"], rel=1e-12)
    for prec in (1, 3):
        s1, l1 = runs[prec]
        assert s1["termination_type"] != "FAILURE"
        assert s1["final_cost"] == pytest.approx(s0["final_cost"], rel=1e-6)
        assert s1["final_cost"] != s0["final_cost"]   # the rounding is really applied
    assert runs[3][0]["final_cost"] != runs[1][0]["final_cost"]   # another rounding


# ---------------------------------------------------------------------------
# HIP path vs oracle (GPU)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def solver():
    from bundleadjustment_amd import Solver
    s = Solver(0)
    yield s
    s.close()


def gpu_solve(solver, p, **kw):
    solver.set_problem(p)
    summ = solver.solve(Options(linear_solver_type="ITERATIVE_SCHUR", **kw))
    cams, pts = solver.params()
    return cams, pts, summ, solver.iteration_log()


def compare(glog, olog, n, rtol=1e-9):
    assert len(glog) >= n and len(olog) >= n, (len(glog), len(olog))
    for g, o in zip(glog[:n], olog[:n]):
        assert g["step_is_valid"] == o["step_is_valid"], (g, o)
        assert g["step_is_successful"] == o["step_is_successful"], (g, o)
        if g["iteration"] > 0:
            assert g["linear_solver_iterations"] == o["linear_solver_iterations"], (g["iteration"], g, o)
        assert g["cost"] == pytest.approx(o["cost"], rel=rtol), (g["iteration"], g["cost"], o["cost"])
        assert g["trust_region_radius"] == pytest.approx(o["trust_region_radius"], rel=1e-9)


# matvec forms of the implicit Schur complement: "auto" the solver's choice
# by size (point-aligned chunks over the 16-value rank-2 records W_o = c'Z
# with the per-observation products t_o = W_o v_p); "gather" the point-major
# 18-value W gathered in camera order (BA_PCG_T=0); "t_gather" the products
# forced on (BA_PCG_T=1); "pairs" the value-pair point passes k_pcg_point /
# k_pcg_point_t instead of the point-aligned chunks (BA_PCG_SEG=0,
# BA_PCG_T=1); "w18" the point-aligned chunks over the 18-value W records
# (BA_PCG_PC=0)
MATVECS = ["auto", "gather", "t_gather", "pairs", "w18"]
# the matvec forms that run on the rank-2 records (oracle precision 3 with
# fp32 W; the others round the 18 W entries: precision 1)
RANK2 = {"auto", "t_gather"}


def set_matvec(monkeypatch, mode):
    if mode == "w18":
        monkeypatch.setenv("BA_PCG_PC", "0")
    elif mode != "auto":
        monkeypatch.setenv("BA_PCG_T", "0" if mode == "gather" else "1")
        if mode == "pairs":
            monkeypatch.setenv("BA_PCG_SEG", "0")


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["FP64", "MIXED_FP32"])
@pytest.mark.parametrize("cfg,scale", [("c3", 0.01), ("c4", 0.01)])
def test_gpu_rank2_pcg_records_track_the_full_records(solver, cfg, scale, precision, monkeypatch):
    """The PCG point pass over the 16-value rank-2 records (k_obs_w_rc<.., PC>:
    W_o = c^T Z with c's four nonzero translation entries; the default where
    it applies) against the 18-value records (BA_PCG_PC=0): the same products
    up to rounding (they associate differently), so fp64 costs to 1e-10 and
    the same CG counts — at <= 200 cameras (LDS camera table) and beyond (the
    DMA-gathered camera records).  fp32 W rounds c and Z instead of their
    product: costs to 1e-6 there."""
    p = make_config(cfg, scale=scale)
    kw = dict(preconditioner_type="SCHUR_JACOBI", max_num_iterations=6, precision=precision)
    ca, xa, sa, la = gpu_solve(solver, p, **kw)
    monkeypatch.setenv("BA_PCG_PC", "0")
    cb, xb, sb, lb = gpu_solve(solver, p, **kw)
    rel = 1e-10 if precision == "FP64" else 1e-6
    assert len(la) == len(lb)
    for a, b in zip(la, lb):
        assert a["cost"] == pytest.approx(b["cost"], rel=rel)
    if precision == "FP64":
        assert [r["linear_solver_iterations"] for r in la] == [r["linear_solver_iterations"] for r in lb]
    assert sa.final_cost == pytest.approx(sb.final_cost, rel=rel)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["FP64", "MIXED_FP32"])
@pytest.mark.parametrize("shape", ["c4", "many"])
def test_gpu_jfree_pcg_point_pass_is_bitwise_the_record_pass(solver, shape, precision, monkeypatch):
    """Beyond the LDS camera table the PCG point pass forms the rank-2
    records itself (k_pcg_point_jf, no W written or read) — the values
    k_obs_w_rc<.., PC> stores (rounded to fp32 with MIXED_FP32), the record
    and its products through the same contraction-free helpers (pc_record,
    pc_v, pc_t) as the record-reading pair of passes (BA_PCG_JF=0).  lin_obs
    is inlined into a different kernel, where the compiler may contract its
    products into FMAs differently: the solves agree to rounding (costs
    1e-12, parameters 1e-9) with the same CG counts and decisions."""
    p = make_config("c4", scale=0.01) if shape == "c4" else make_synthetic(1300, 4000, obs_per_pt=4, seed=21)
    kw = dict(preconditioner_type="SCHUR_JACOBI", max_num_iterations=6, precision=precision)
    monkeypatch.setenv("BA_PCG_JF", "1")   # (the fp64 default; fp32 W keeps the records by default)
    ca, xa, sa, la = gpu_solve(solver, p, **kw)
    monkeypatch.setenv("BA_PCG_JF", "0")
    cb, xb, sb, lb = gpu_solve(solver, p, **kw)
    assert sa.final_cost == pytest.approx(sb.final_cost, rel=1e-12)
    np.testing.assert_allclose(ca, cb, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(xa, xb, rtol=1e-9, atol=1e-12)
    assert len(la) == len(lb)
    for a, b in zip(la, lb):
        assert a["cost"] == pytest.approx(b["cost"], rel=1e-12)
        assert a["linear_solver_iterations"] == b["linear_solver_iterations"]
        assert a["step_is_successful"] == b["step_is_successful"]
    print("max |dcam| %.3g  max |dpt| %.3g" % (np.abs(ca - cb).max(), np.abs(xa - xb).max()))


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["FP64", "MIXED_FP32"])
@pytest.mark.parametrize("shape", ["c3", "c4", "resets"])
def test_gpu_point_step_from_accumulated_cg_products(solver, shape, precision, monkeypatch):
    """ITERATIVE_SCHUR back substitution from the CG's accumulated point
    products (vacc = sum_k alpha_k vpt(p_k) = vpt(y), k_pcg_vacc; reset to
    vpt(y) at each residual reset) and the block form of the model cost change
    (g'd + d'Hd/2 from Hcc, Hpp and vacc), against the per-observation J form
    (BA_PCG_PACC=0): the same quantities up to rounding — costs 1e-11, radii
    1e-9, identical decisions and CG counts, parameters 1e-8.  MIXED_FP32: the
    accumulated products carry the stored fp32 blocks into the back
    substitution (the J form stays fp64), a relative ~1e-7 perturbation of the
    point step: costs 1e-9, radii 1e-7, parameters 1e-6."""
    if shape == "resets":
        p = make_config("c2", scale=0.2)
        kw = dict(preconditioner_type="JACOBI", max_num_iterations=4, eta=1e-14, max_linear_solver_iterations=23)
    else:
        p = make_config(shape, scale=0.01)
        kw = dict(preconditioner_type="SCHUR_JACOBI", max_num_iterations=8)
    kw["precision"] = precision
    ca, xa, sa, la = gpu_solve(solver, p, **kw)
    monkeypatch.setenv("BA_PCG_PACC", "0")
    cb, xb, sb, lb = gpu_solve(solver, p, **kw)
    if shape == "resets":
        assert max(r["linear_solver_iterations"] for r in la[1:]) == 23
    f64 = precision == "FP64"
    assert len(la) == len(lb)
    for a, b in zip(la, lb):
        assert a["step_is_successful"] == b["step_is_successful"]
        assert a["linear_solver_iterations"] == b["linear_solver_iterations"]
        assert a["cost"] == pytest.approx(b["cost"], rel=1e-11 if f64 else 1e-9)
        assert a["trust_region_radius"] == pytest.approx(b["trust_region_radius"], rel=1e-9 if f64 else 1e-7)
    assert sa.final_cost == pytest.approx(sb.final_cost, rel=1e-11 if f64 else 1e-9)
    np.testing.assert_allclose(ca, cb, rtol=1e-8 if f64 else 1e-6, atol=1e-10 if f64 else 1e-8)
    np.testing.assert_allclose(xa, xb, rtol=1e-8 if f64 else 1e-6, atol=1e-10 if f64 else 1e-8)


@pytest.mark.gpu
@pytest.mark.parametrize("pc", PRECONDITIONERS)
@pytest.mark.parametrize("cfg,scale", [("c1", 1.0), ("c2", 0.2), ("c3", 0.01)])
@pytest.mark.parametrize("mv", MATVECS)
def test_gpu_iterative_matches_oracle(solver, oracle_lib, cfg, scale, pc, mv, monkeypatch):
    """Every matvec form against the oracle."""
    set_matvec(monkeypatch, mv)
    p = make_config(cfg, scale=scale)
    _, _, so, olog = oracle_lib.solve(p, oracle_opts(oracle_lib, pc, max_num_iterations=8))
    _, _, sg, glog = gpu_solve(solver, p, preconditioner_type=pc, max_num_iterations=8)
    compare(glog, olog, min(len(glog), len(olog), 6))
    assert sg.final_cost == pytest.approx(so["final_cost"], rel=1e-8)


@pytest.mark.gpu
@pytest.mark.parametrize("pc", PRECONDITIONERS)
def test_gpu_iterative_reaches_dense_minimum(solver, pc):
    p = gauge_fixed("c3", 0.05)
    solver.set_problem(p)
    sd = solver.solve(Options(max_num_iterations=100, function_tolerance=1e-12))
    _, _, si, _ = gpu_solve(solver, p, preconditioner_type=pc, max_num_iterations=100, function_tolerance=1e-12)
    assert si.termination_type != "FAILURE"
    assert si.final_cost == pytest.approx(sd.final_cost, rel=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("mv", MATVECS)
def test_gpu_iterative_residual_reset_and_cap(solver, oracle_lib, mv, monkeypatch):
    """Residual resets (r = b - S x every 10 CG iterations: a matvec of the
    iterate) and the iteration cap, on every matvec form."""
    set_matvec(monkeypatch, mv)
    p = make_config("c2", scale=0.2)
    kw = dict(max_num_iterations=4, eta=1e-14, max_linear_solver_iterations=23)
    _, _, so, olog = oracle_lib.solve(p, oracle_opts(oracle_lib, "JACOBI", **kw))
    _, _, sg, glog = gpu_solve(solver, p, preconditioner_type="JACOBI", **kw)
    assert max(r["linear_solver_iterations"] for r in glog[1:]) == 23
    compare(glog, olog, len(olog), rtol=1e-8)


@pytest.mark.gpu
def test_gpu_iterative_duplicate_observations(solver, oracle_lib):
    p = with_duplicate_observations(make_config("c2", scale=0.2))
    _, _, so, olog = oracle_lib.solve(p, oracle_opts(oracle_lib, "SCHUR_JACOBI", max_num_iterations=6))
    _, _, sg, glog = gpu_solve(solver, p, preconditioner_type="SCHUR_JACOBI", max_num_iterations=6)
    compare(glog, olog, min(len(glog), len(olog)))


@pytest.mark.gpu
def test_gpu_iterative_is_deterministic(solver):
    p = make_config("c3", scale=0.05)
    c1, x1, s1, _ = gpu_solve(solver, p, preconditioner_type="SCHUR_JACOBI", max_num_iterations=5)
    c2, x2, s2, _ = gpu_solve(solver, p, preconditioner_type="SCHUR_JACOBI", max_num_iterations=5)
    assert s1.final_cost == s2.final_cost
    assert np.array_equal(c1, c2) and np.array_equal(x1, x2)


@pytest.mark.gpu
def test_gpu_iterative_grid_path_is_deterministic(solver):
    """> 256 cameras (thread-per-camera grid kernels, many workgroups per
    CG step): repeated solves are bitwise identical.  Guards the hand-off of
    rho / Q0 between CG iterations (the lead workgroup writes the next
    iteration's values into the other parity slot while the other workgroups
    of the same launch still read the current ones)."""
    p = make_synthetic(6000, 6000, obs_per_pt=4, seed=5)
    runs = [gpu_solve(solver, p, preconditioner_type="JACOBI", max_num_iterations=4,
                      max_linear_solver_iterations=30, eta=1e-6) for _ in range(4)]
    c0, x0, s0, l0 = runs[0]
    assert any(r["linear_solver_iterations"] > 3 for r in l0[1:])
    for c, x, s, l in runs[1:]:
        assert s.final_cost == s0.final_cost
        assert np.array_equal(c, c0) and np.array_equal(x, x0)
        assert [r["linear_solver_iterations"] for r in l] == [r["linear_solver_iterations"] for r in l0]


@pytest.mark.gpu
def test_gpu_iterative_motion_only_and_no_cameras(solver, oracle_lib):
    """Edge cases: motion-only (no eliminated points: S = F'F + D^2) and
    structure-only (every camera fixed: empty reduced system)."""
    p = make_config("f2f")
    _, _, so, olog = oracle_lib.solve(p, oracle_opts(oracle_lib, "SCHUR_JACOBI", max_num_iterations=10))
    _, _, sg, glog = gpu_solve(solver, p, preconditioner_type="SCHUR_JACOBI", max_num_iterations=10)
    compare(glog, olog, min(len(glog), len(olog)))
    q = make_synthetic(3, 200, obs_per_pt=3, seed=11)
    for c in range(3):
        bp.fix_camera(q, c)
    _, _, so, olog = oracle_lib.solve(q, oracle_opts(oracle_lib, "JACOBI", max_num_iterations=10))
    _, _, sg, glog = gpu_solve(solver, q, max_num_iterations=10)
    assert sg.final_cost == pytest.approx(so["final_cost"], rel=1e-9)


@pytest.mark.gpu
def test_gpu_iterative_rejects_bad_options(solver):
    from bundleadjustment_amd._native import BAError
    solver.set_problem(make_config("c1"))
    with pytest.raises(BAError):
        solver.solve(Options(linear_solver_type="ITERATIVE_SCHUR", max_linear_solver_iterations=0))


@pytest.mark.gpu
@pytest.mark.parametrize("pc", PRECONDITIONERS)
def test_gpu_iterative_many_cameras(solver, oracle_lib, pc):
    """> 256 variable cameras: the camera side runs as thread-per-camera grid
    kernels (k_pcg_q / k_pcg_xr / k_pcg_p) instead of one workgroup; the
    per-camera gathers use one slice per camera."""
    p = make_synthetic(1300, 4000, obs_per_pt=4, seed=21)
    _, _, so, olog = oracle_lib.solve(p, oracle_opts(oracle_lib, pc, max_num_iterations=6))
    _, _, sg, glog = gpu_solve(solver, p, preconditioner_type=pc, max_num_iterations=6)
    compare(glog, olog, len(olog))
    kw = dict(max_num_iterations=3, eta=1e-14, max_linear_solver_iterations=21)   # residual resets
    _, _, so, olog = oracle_lib.solve(p, oracle_opts(oracle_lib, pc, **kw))
    _, _, sg, glog = gpu_solve(solver, p, preconditioner_type=pc, **kw)
    compare(glog, olog, len(olog), rtol=1e-8)


@pytest.mark.gpu
@pytest.mark.parametrize("pc", PRECONDITIONERS)
def test_gpu_mixed_fp32_matches_fp64(solver, pc):
    """BA_MIXED_FP32 (fp32 storage of the per-observation Schur blocks W):
    final cost within 1e-6 relative of the fp64 path, and the
    iterations track the fp64 ones."""
    p = gauge_fixed("c3", 0.05)
    kw = dict(preconditioner_type=pc, max_num_iterations=40, function_tolerance=1e-10)
    _, _, s64, log64 = gpu_solve(solver, p, **kw)
    c32, x32, s32, log32 = gpu_solve(solver, p, precision="MIXED_FP32", **kw)
    assert s32.termination_type != "FAILURE"
    assert s32.final_cost == pytest.approx(s64.final_cost, rel=1e-6)
    for g, o in list(zip(log32, log64))[:4]:
        assert g["cost"] == pytest.approx(o["cost"], rel=1e-6)
    # deterministic as well
    c32b, x32b, s32b, _ = gpu_solve(solver, p, precision="MIXED_FP32", **kw)
    assert s32b.final_cost == s32.final_cost and np.array_equal(c32, c32b) and np.array_equal(x32, x32b)


@pytest.mark.gpu
@pytest.mark.parametrize("pc", PRECONDITIONERS)
@pytest.mark.parametrize("cfg,scale", [("c2", 0.2), ("c3", 0.01), ("c4", 0.01)])
@pytest.mark.parametrize("mv", MATVECS)
def test_gpu_mixed_fp32_matches_oracle_mixed(solver, oracle_lib, cfg, scale, pc, mv, monkeypatch):
    """BA_MIXED_FP32 against the oracle's independent fp32 restatement: the
    18 W entries rounded to float in the matvec (oracle precision 1), or for
    the forms on the 16-value rank-2 records c and Z rounded to float and
    associated as Z'(c x), c'(Z v) (precision 3); the rhs and the
    preconditioner from the rounded W entries, the back substitution in fp64
    (the GPU's from the accumulated products of the stored fp32 blocks, a
    relative ~1e-7 perturbation of the point step).
    The iterations match like the fp64 ones — cost 1e-9, identical decisions
    and CG counts — on every matvec form (mv "pairs" runs
    k_pcg_point_t<float>)."""
    set_matvec(monkeypatch, mv)
    p = make_config(cfg, scale=scale)
    prec = 3 if mv in RANK2 else 1
    _, _, so, olog = oracle_lib.solve(p, oracle_opts(oracle_lib, pc, max_num_iterations=8, precision=prec))
    _, _, sg, glog = gpu_solve(solver, p, preconditioner_type=pc, max_num_iterations=8, precision="MIXED_FP32")
    compare(glog, olog, min(len(glog), len(olog), 6))
    assert sg.final_cost == pytest.approx(so["final_cost"], rel=1e-8)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_gpu_pcg_t_auto_threshold(solver, monkeypatch):
    """2M observations: the fp64 W (144 B/obs = 288 MB) outgrows the 256-MiB
    Infinity Cache, so the solver picks the per-observation product matvec by
    itself; it must match the W-gather matvec (BA_PCG_T=0) on the same
    problem: costs 1e-10, identical decisions and CG counts."""
    p = make_config("c3", scale=2.0)
    assert 144 * p.n_obs > 256 * 2 ** 20
    kw = dict(preconditioner_type="SCHUR_JACOBI", max_num_iterations=5)
    _, _, sa, la = gpu_solve(solver, p, **kw)
    monkeypatch.setenv("BA_PCG_T", "0")
    _, _, sb, lb = gpu_solve(solver, p, **kw)
    compare(la, lb, len(lb), rtol=1e-10)
    assert sa.final_cost == pytest.approx(sb.final_cost, rel=1e-10)


@pytest.mark.gpu
def test_gpu_mixed_fp32_requires_iterative(solver):
    from bundleadjustment_amd._native import BAError
    solver.set_problem(make_config("c1"))
    with pytest.raises(BAError):
        solver.solve(Options(precision="MIXED_FP32"))


@pytest.mark.gpu
@pytest.mark.parametrize("solver_type", ["DENSE_SCHUR", "ITERATIVE_SCHUR"])
@pytest.mark.parametrize("dups", [False, True])
def test_gpu_exchange_path_on_one_rank(solver_type, dups, monkeypatch):
    """The multi-GPU exchange path (RCCL all-reduces of the camera blocks,
    the packed lower triangle of S, the CG matvec slices, the step scalars)
    forced on a one-rank communicator, where every all-reduce is the identity:
    results are bitwise those of the communicator-free solve.  Without
    duplicate observations the single-rank dense path adds the LM diagonal
    inside the Schur-diagonal fold; with them (diagonal pair blocks) after
    k_schur_pairs, as the exchange path does."""
    from bundleadjustment_amd import Solver
    p = make_config("c2", scale=0.2)
    if dups:
        p = with_duplicate_observations(p)
    opts = Options(linear_solver_type=solver_type, preconditioner_type="SCHUR_JACOBI", max_num_iterations=6)
    with Solver(0) as s0:
        s0.set_problem(p)
        r0 = s0.solve(opts)
        c0, x0 = s0.params()
    monkeypatch.setenv("BA_FORCE_COLLECTIVES", "1")
    with Solver(0) as s1:
        s1.comm_init(Solver.unique_id(), 1, 0)
        s1.set_problem(p)
        r1 = s1.solve(opts)
        c1, x1 = s1.params()
    assert r1.final_cost == r0.final_cost and r1.num_iterations == r0.num_iterations
    assert np.array_equal(c0, c1) and np.array_equal(x0, x1)
