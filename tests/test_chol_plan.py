"""The split Cholesky's task schedule (bundleadjustment_amd/csrc/ba_chol_split.hip
chol_split_plan / chol_flow_tasks), checked on the host: tools/chol_plan_check
replays the per-step task tables and the flow form's one list for every order
up to 40 block columns (ranks 1 and 4) — every tile receives every panel
exactly once, in order, after the panel exists and before the tile is due; no
two tasks of one launch touch one tile; the flow list never makes a task wait
on one after it, and the chain workgroup can always advance."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
def test_split_cholesky_schedule_invariants(tmp_path):
    exe = tmp_path / "chol_plan_check"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-std=c++17", "-I",
                    os.path.join(ROOT, "bundleadjustment_amd", "csrc"),
                    os.path.join(ROOT, "tools", "chol_plan_check.hip"), "-o", str(exe)],
                   check=True, capture_output=True, timeout=300)
    out = subprocess.run([str(exe), "quick"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:]
    assert "0 violations" in out.stdout
