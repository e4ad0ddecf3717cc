"""Diagnostics of the overlapped DENSE_SCHUR form (ba_chol_persist.hip OvArgs):
the reduced system of C3 formed N times by the separate pair / diagonal / fold
launches and N times by the overlapped launch with the factorisation switched
off (BA_DEBUG_OV_PASS=1), for a rocprofv3 kernel trace of both."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bundleadjustment_amd import Solver, make_config  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
p = make_config("c3")
with Solver(0) as s:
    s.set_problem(p)
    for _ in range(n):
        s.debug_blocks(1e4, with_s=False)
    os.environ["BA_DEBUG_OV_PASS"] = "1"
    for _ in range(n):
        s.debug_blocks(1e4, with_s=False)
print("done")
