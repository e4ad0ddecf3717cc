"""Build C-ABI problems from the golden functor fixtures (tests/golden/functors.npz):
one observation per (camera, point) case, for each of the reference's three
functors (Optimizer.h:49-194)."""
import numpy as np

from bundleadjustment_amd.problem import Problem


def golden_problem(g, kind: str, huber_a: float = 0.0) -> Problem:
    m = g["cams"].shape[0]
    idx = np.arange(m, dtype=np.int32)
    cams = g["cams"].copy()
    pts = g["pts"].copy()
    cam_fixed = np.zeros(m, np.uint8)
    pt_fixed = np.zeros(m, np.uint8)
    if kind == "angle":
        pass
    elif kind == "pose":           # PoseOnlyAngleReprojectionError: constant float point
        pt_fixed[:] = 1
        pts = pts.astype(np.float32).astype(np.float64)
    elif kind == "point":          # PointOnlyReprojectionError: constant float extrinsic
        cam_fixed[:] = 1
    else:
        raise ValueError(kind)
    return Problem(cams=cams, K=g["K"].copy(), pts=pts, obs_cam=idx, obs_pt=idx.copy(), obs_uv=g["uv"].copy(),
                   cam_fixed=cam_fixed, cam_fixed_extr=g["extr"].copy(), pt_fixed=pt_fixed,
                   huber_a=huber_a).normalized()


def golden_expected(g, kind: str):
    """(r, J[n,2,9]) in the ABI layout (camera 6 | point 3)."""
    m = g["cams"].shape[0]
    J = np.zeros((m, 2, 9))
    if kind == "angle":
        return g["r_angle"], g["J_angle"]
    if kind == "pose":
        J[:, :, :6] = g["J_pose"]
        return g["r_pose"], J
    J[:, :, 6:] = g["J_pt"]
    return g["r_pt"], J
