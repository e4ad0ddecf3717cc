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
