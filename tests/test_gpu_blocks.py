"""The blocks the J-free kernels form, read directly (ba_debug_blocks), against
the oracle.

The per-observation r / J parity test (test_gpu_parity.py) reads the JR
records of ba_linearize's read-back kernel; the timed iteration never stores
J.  Here the outputs of the kernels a solve actually runs are compared:

  Hpp, gp  k_lin_point (r, J, Huber and the point blocks in one pass)
  Hcc, gc  k_cam_assemble_rc (camera-major, J recomputed)
  S, rhs   k_point_elim + k_obs_w_rc (compact 128-B records up to 200
           cameras, 18-double W beyond) + k_cam_schur_diag(_c) +
           k_schur_pairs(_c) + the LM diagonal: the reduced camera system as
           the Cholesky receives it (ceres' SchurComplementSolver,
           Optimizer.cpp:242)

against sums of the oracle's corrected per-observation Jacobians (Hpp, gp,
Hcc, gc) and the oracle's own DENSE_SCHUR assembly (oracle.reduced_system,
iteration-0 Jacobi scaling, the same radius).  Configs: C3 at full size (200
cameras: LDS camera tables, compact W) and the C4 shard (1000 cameras: the
global table gtbl, 18-double W, the split-path system of 5994 rows).

Tolerances: the blocks are sums of ~10 (points) or ~5000 (cameras) products
in a different order: 1e-11 relative to each array's largest entry.  S is a
difference (s Hcc s + D^2 - sum W W^T) whose entries cancel: 1e-10 of the
largest |S| entry, 1e-11 relative on the diagonal; rhs likewise.
"""
import numpy as np
import pytest

from bundleadjustment_amd import Solver, make_config

pytestmark = pytest.mark.gpu


def oracle_blocks(oracle_lib, p):
    """Hpp (xx, xy, xz, yy, yz, zz), gp, Hcc (lower row-major), gc from the
    oracle's corrected r and J (caller order)."""
    r, J, _, ok = oracle_lib.linearize(p)
    assert ok
    Jc, Jp = J[:, :, :6], J[:, :, 6:]
    hp = np.einsum("oia,oib->oab", Jp, Jp)
    gpo = np.einsum("oia,oi->oa", Jp, r)
    hc = np.einsum("oia,oib->oab", Jc, Jc)
    gco = np.einsum("oia,oi->oa", Jc, r)
    Hpp = np.zeros((p.n_pts, 3, 3))
    gp = np.zeros((p.n_pts, 3))
    Hcc = np.zeros((p.n_cams, 6, 6))
    gc = np.zeros((p.n_cams, 6))
    np.add.at(Hpp, p.obs_pt, hp)
    np.add.at(gp, p.obs_pt, gpo)
    np.add.at(Hcc, p.obs_cam, hc)
    np.add.at(gc, p.obs_cam, gco)
    iu = [(0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2)]
    Hpp6 = np.stack([Hpp[:, a, b] for a, b in iu], axis=1)
    tri = [(a, b) for a in range(6) for b in range(a + 1)]
    Hcc21 = np.stack([Hcc[:, a, b] for a, b in tri], axis=1)
    return Hpp6, gp, Hcc21, gc


def close_to_scale(got, ref, rel, what):
    scale = max(np.abs(ref).max(), 1e-300)
    err = np.abs(got - ref).max()
    assert err <= rel * scale, f"{what}: max |diff| {err:.3e} > {rel:g} x {scale:.3e}"


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg,scale", [("c3", 1.0), ("c4", 0.125)])
def test_jfree_blocks_and_reduced_system_match_oracle(oracle_lib, cfg, scale):
    p = make_config(cfg, scale=scale)
    radius = 1e4
    with Solver(0) as s:
        s.set_problem(p)
        got = s.debug_blocks(radius)
    Hpp, gp, Hcc, gc = oracle_blocks(oracle_lib, p)
    close_to_scale(got["Hpp"], Hpp, 1e-11, "Hpp")
    close_to_scale(got["gp"], gp, 1e-11, "gp")
    close_to_scale(got["Hcc"], Hcc, 1e-11, "Hcc")
    close_to_scale(got["gc"], gc, 1e-11, "gc")
    lhs, rhs = oracle_lib.reduced_system(p, radius=radius)
    n = got["n"]
    assert lhs.shape == (n, n) and got["S"].shape == (n, n)
    tril = np.tril_indices(n)
    close_to_scale(got["S"][tril], lhs[tril], 1e-10, "S (lower)")
    d = np.arange(n)
    assert np.allclose(got["S"][d, d], lhs[d, d], rtol=1e-11, atol=0), "S diagonal"
    close_to_scale(got["rhs"], rhs, 1e-10, "rhs")



@pytest.mark.timeout(600)
def test_diagonal_slices_in_the_pair_launch_are_bitwise_the_separate_launch(monkeypatch):
    """C3 (compact W records): the diagonal Schur slices ride in the pair
    pass's launch by default (one wave per camera slice, wave_sum); with
    BA_DIAG_IN_PAIRS=0 they run as k_cam_schur_diag_cd (one 64-thread
    workgroup per slice, block_sum) and the fold rides in the pair launch
    instead.  Both reductions add the same lane values in the same tree, so
    the reduced system and its rhs are bitwise equal."""
    p = make_config("c3", scale=1.0)
    with Solver(0) as s:
        s.set_problem(p)
        a = s.debug_blocks(1e4)
        monkeypatch.setenv("BA_DIAG_IN_PAIRS", "0")
        b = s.debug_blocks(1e4)
    n = a["n"]
    tril = np.tril_indices(n)
    assert np.array_equal(a["S"][tril], b["S"][tril])
    assert np.array_equal(a["rhs"], b["rhs"])


@pytest.mark.timeout(600)
def test_overlapped_pass_is_bitwise_the_separate_passes(monkeypatch):
    """C3: the reduced system the overlapped factorisation forms inside its
    own launch (ba_chol_persist.hip OvArgs: per-XCD queues of wave-sized work
    items in tile-column order — pair blocks with two LDS-DMA rounds in
    flight, diagonal slices, the fold by the wave that completes a camera)
    is bitwise the reduced system of the separate pair / diagonal / fold
    launches: the same lanes, pairs, products and reductions per entry.
    BA_DEBUG_OV_PASS=1 makes ba_debug_blocks run that launch with the
    factorisation switched off (and fail if the form does not apply)."""
    p = make_config("c3", scale=1.0)
    with Solver(0) as s:
        s.set_problem(p)
        a = s.debug_blocks(1e4)
        monkeypatch.setenv("BA_DEBUG_OV_PASS", "1")
        b = s.debug_blocks(1e4)
        c = s.debug_blocks(3e2)    # a second launch: cumulative counters and tickets
        monkeypatch.delenv("BA_DEBUG_OV_PASS")
        d = s.debug_blocks(3e2)
    n = a["n"]
    tril = np.tril_indices(n)
    assert np.array_equal(a["S"][tril], b["S"][tril])
    assert np.array_equal(a["rhs"], b["rhs"])
    assert np.array_equal(c["S"][tril], d["S"][tril])
    assert np.array_equal(c["rhs"], d["rhs"])


@pytest.mark.timeout(900)
def test_many_camera_dma_pairs_are_bitwise_the_register_pairs(monkeypatch):
    """The C4 shard (1000 cameras): the pair pass gathers the compact records
    by LDS-DMA with each block's camera constants in registers (the LDS
    camera table does not fit beside the DMA buffers), and the diagonal
    slices ride in its launch on the same DMA buffers (pairs_take_diag_nt);
    BA_DIAG_IN_PAIRS=0 keeps their separate launch, BA_PAIRS_DMA=0 the
    per-lane register gathers with the table in LDS and the separate
    diagonal launch.  Same lanes, pairs, products and reductions: the reduced
    system is bitwise the same in all three."""
    p = make_config("c4", scale=0.125)
    with Solver(0) as s:
        s.set_problem(p)
        a = s.debug_blocks(1e4)
        monkeypatch.setenv("BA_DIAG_IN_PAIRS", "0")
        c = s.debug_blocks(1e4)
        monkeypatch.delenv("BA_DIAG_IN_PAIRS")
        monkeypatch.setenv("BA_PAIRS_DMA", "0")
        b = s.debug_blocks(1e4)
    n = a["n"]
    tril = np.tril_indices(n)
    for other in (b, c):
        assert np.array_equal(a["S"][tril], other["S"][tril])
        assert np.array_equal(a["rhs"], other["rhs"])
