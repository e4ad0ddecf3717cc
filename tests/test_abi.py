"""CPU tests of the C-ABI boundary (include/ba_hip.h): the library loads,
exports every declared symbol, and the ctypes mirrors match the C layout.
No compute calls (no GPU here)."""
import ctypes as C
import re
import subprocess

import pytest

from bundleadjustment_amd import _native as N
from conftest import ROOT

HEADER = ROOT / "include" / "ba_hip.h"


def declared_functions():
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ba_[a-z_]+)\s*\(", txt)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    for f in ("ba_create", "ba_destroy", "ba_set_problem", "ba_solve", "ba_get_params", "ba_eval_residuals",
              "ba_last_error", "ba_comm_init"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    lib = N.load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (ba_[a-z_]+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    for f in declared_functions():
        assert hasattr(lib, f)
    assert {name for name, _, _ in N.SIGNATURES} == set(declared_functions())
    assert lib.ba_abi_version() == N.BA_ABI_VERSION == 2


def test_default_options_are_ceres_defaults():
    o = N.default_options()
    assert o.max_num_iterations == 50 and o.max_num_consecutive_invalid_steps == 5 and o.jacobi_scaling == 1
    assert (o.function_tolerance, o.gradient_tolerance, o.parameter_tolerance) == (1e-6, 1e-10, 1e-8)
    assert (o.initial_trust_region_radius, o.max_trust_region_radius) == (1e4, 1e16)
    assert (o.min_relative_decrease, o.min_lm_diagonal, o.max_lm_diagonal) == (1e-3, 1e-6, 1e32)


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "ba_hip.h"
#define F(T, f) printf("%s.%s %zu\n", #T, #f, offsetof(T, f));
int main(void) {
  printf("ba_problem %zu\nba_options %zu\nba_summary %zu\nba_iteration %zu\n", sizeof(ba_problem),
         sizeof(ba_options), sizeof(ba_summary), sizeof(ba_iteration));
  F(ba_problem, cams) F(ba_problem, obs_uv) F(ba_problem, huber_a)
  F(ba_options, function_tolerance) F(ba_options, max_lm_diagonal) F(ba_options, preconditioner_type)
  F(ba_options, eta) F(ba_iteration, linear_solver_iterations)
  F(ba_summary, num_iterations) F(ba_summary, termination_type) F(ba_summary, solve_time_s)
  F(ba_iteration, cost) F(ba_iteration, model_cost_change) F(ba_iteration, iteration_time_s)
  printf("ba_prune_problem %zu\n", sizeof(ba_prune_problem));
  F(ba_prune_problem, extr) F(ba_prune_problem, obs_cam) F(ba_prune_problem, obs_dist)
  printf("ba_pose_batch %zu\n", sizeof(ba_pose_batch));
  F(ba_pose_batch, obs_offset) F(ba_pose_batch, pts) F(ba_pose_batch, obs_uv) F(ba_pose_batch, huber_a)
  return 0;
}
"""


def test_ctypes_layout_matches_c_compiler(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    vals = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                          check=True).stdout.splitlines())
    types = {"ba_problem": N.ba_problem, "ba_options": N.ba_options, "ba_summary": N.ba_summary,
             "ba_iteration": N.ba_iteration, "ba_prune_problem": N.ba_prune_problem,
             "ba_pose_batch": N.ba_pose_batch}
    for k, v in vals.items():
        if "." in k:
            t, f = k.split(".")
            assert getattr(types[t], f).offset == int(v), k
        else:
            assert C.sizeof(types[k]) == int(v), k


def test_errors_without_gpu_are_reported_not_raised():
    """ba_create on a machine without a usable device returns a status (no abort)."""
    lib = N.load_library()
    h = C.c_void_p()
    st = lib.ba_create(C.byref(h), 10_000)
    assert st != N.BA_OK
    assert lib.ba_destroy(None) == N.BA_OK
    assert lib.ba_set_problem(None, None) == 1


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(N.NativeLibraryError):
        N.load_library(tmp_path / "nope.so")
