import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")
    config.addinivalue_line("markers", "slow: larger sizes")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def golden():
    return np.load(GOLDEN / "functors.npz")


def rel_err(a, b, floor=1e-300):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.max(np.abs(a - b) / np.maximum(np.maximum(np.abs(a), np.abs(b)), floor))


def assert_close(a, b, rtol, atol, what=""):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = np.abs(a - b)
    tol = atol + rtol * np.maximum(np.abs(a), np.abs(b))
    bad = err > tol
    if np.any(bad):
        i = np.unravel_index(np.argmax(err - tol), a.shape)
        raise AssertionError(f"{what}: {bad.sum()} / {a.size} entries out of tolerance "
                             f"(rtol={rtol}, atol={atol}); worst at {i}: {a[i]!r} vs {b[i]!r}")


def compare_logs(glog, olog, rtol_cost=1e-10, n=None, strict_iters=None, late_rtol=1e-7):
    """Iteration-by-iteration comparison of the ceres IterationSummary fields.
    `strict_iters`: compare costs at rtol_cost only for the first iterations
    and at late_rtol afterwards (problems with a free gauge: rounding
    differences drift along the null space)."""
    n = n or min(len(glog), len(olog))
    assert len(glog) >= n and len(olog) >= n
    for g, o in zip(glog[:n], olog[:n]):
        tol = rtol_cost if strict_iters is None or g["iteration"] < strict_iters else late_rtol
        assert g["iteration"] == o["iteration"]
        assert g["step_is_valid"] == o["step_is_valid"], (g, o)
        assert g["step_is_successful"] == o["step_is_successful"], (g, o)
        assert g["cost"] == pytest.approx(o["cost"], rel=tol), (g["iteration"], g["cost"], o["cost"])
        assert g["trust_region_radius"] == pytest.approx(o["trust_region_radius"], rel=1e-9)
        if g["step_is_valid"] and g["iteration"] > 0:
            # the model cost change is a small difference of quadratic-model
            # terms near convergence: relative accuracy ~cond(S)*eps (observed
            # <= 3e-8); it only enters the accept test rho > 1e-3.
            mt = 1e-6 if tol == rtol_cost else 1e-3
            assert g["model_cost_change"] == pytest.approx(o["model_cost_change"], rel=mt)
            assert g["relative_decrease"] == pytest.approx(o["relative_decrease"], rel=mt, abs=1e-9)
