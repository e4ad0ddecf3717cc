"""Overlapped DENSE_SCHUR step against the serial forms on one problem:
per-iteration cost / validity and the final parameters (bitwise)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bundleadjustment_amd import Options, Solver, make_config  # noqa: E402
from bundleadjustment_amd import problem as bp  # noqa: E402

cfg, scale, fix = (sys.argv[1], float(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else ("c3", 0.05, 1)
p = make_config(cfg, scale=scale)
if fix:
    bp.fix_camera(p, 1)
runs = {}
for name, env in [("per-step", {"BA_CHOL_PERSIST": "0"}), ("persist serial", {"BA_OVERLAP": "0"}),
                  ("signalled serial", {"BA_OVERLAP": "2"}), ("overlap", {"BA_OVERLAP": "1"}),
                  ("overlap again", {"BA_OVERLAP": "1"})]:
    for k in ("BA_CHOL_PERSIST", "BA_OVERLAP"):
        os.environ.pop(k, None)
    os.environ.update(env)
    with Solver(0) as s:
        s.set_problem(p)
        s.solve(Options(max_num_iterations=6))
        cams, pts = s.params()
        log = s.iteration_log()
    runs[name] = (cams, pts, log)
    print(f"{name:18s}", " ".join(f"{r['cost']:.15e}/{int(r['step_is_valid'])}{int(r['step_is_successful'])}"
                                   for r in log))
ref = runs["per-step"]
for name, (c, q, _) in runs.items():
    print(f"{name:18s} cams equal {np.array_equal(c, ref[0])}  pts equal {np.array_equal(q, ref[1])}  "
          f"max |dcam| {np.max(np.abs(c - ref[0])):.3e}")
