"""Event trace of the overlapped DENSE_SCHUR launch (ba_chol_persist.hip,
BA_OV_TRACE build): tile formation times against the critical workgroup's
steps and the workers' hand-offs.  Build the trace library first:
  make -C bundleadjustment_amd/csrc EXTRA=-DBA_OV_TRACE OBJ=obj_trace OUT=../libba_hip_trace.so
then run  BA_HIP_LIB=bundleadjustment_amd/libba_hip_trace.so python tools/ov_trace.py
(one 2-iteration C3 solve; the trace is the last launch's)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bundleadjustment_amd import Options, Solver, make_config  # noqa: E402
from bundleadjustment_amd import _native  # noqa: E402

p = make_config("c3")
with Solver(0) as s:
    s.set_problem(p)
    s.solve(Options(max_num_iterations=int(os.environ.get("OV_ITERS", "2"))))
lib = _native.load_library()
buf = (C.c_ulonglong * 4096)()
assert lib.ba_debug_ov_trace(buf, 4096) == 0
t = np.array(buf[:], dtype=np.float64)
t0 = t[0]
us = lambda v: (v - t0) / 100.0 if v else float("nan")   # s_memrealtime: 100 MHz
n = 6 * (p.n_cams - 1)
T, TR = (n + 63) // 64, (n + 64) // 64
print(f"n={n} T={T} TR={TR}")
print("step: start  staged   | column c: last tile formed, tiles (c+1,c) (c,c) formed")
for c in range(T):
    col = [us(t[8 + I * T + c]) for I in range(c, TR)]
    print(f"{c:3d}: {us(t[512 + c]):7.1f} {us(t[768 + c]):7.1f}   | {np.nanmax(col):7.1f}  "
          f"{us(t[8 + (c + 1) * T + c]) if c + 1 < TR else float('nan'):7.1f} {us(t[8 + c * T + c]):7.1f}")
g = [us(v) for v in t[1024:1024 + 256]]
print("last item taken (helpers, workers): max %.1f  median %.1f" % (np.nanmax(g), np.nanmedian(g)))
