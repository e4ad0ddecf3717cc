"""The observable output of the reference's BA: the float write-back of
Optimizer.cpp:252-267 —
    R = AngleAxisToRotationMatrix(w)           (double, then .cast<float>())
    t = t.cast<float>()
    extr = [R | t; 0 0 0 1] (Matrix4f), frame->setPose(extr.inverse())
    point->setPosition(X.cast<float>())
— and SURVEY.md §8c's bar for it: the write-back of two solutions is
identical, or within 1 float ulp per entry.  Test helper only."""
import numpy as np

from bundleadjustment_amd import problem as bp


def float_write_back(cams, pts):
    """(R float [C,3,3], t float [C,3], pose float [C,4,4], points float [P,3])."""
    cams = np.asarray(cams, np.float64)
    R = bp.angle_axis_to_rotation(cams[:, :3]).astype(np.float32)
    t = cams[:, 3:].astype(np.float32)
    E = np.zeros((len(cams), 4, 4), np.float32)
    E[:, :3, :3] = R
    E[:, :3, 3] = t
    E[:, 3, 3] = 1.0
    pose = np.linalg.inv(E) if len(cams) else E      # float32 in, float32 out (same routine on both sides)
    return R, t, pose.astype(np.float32), np.asarray(pts, np.float64).astype(np.float32)


def ulp_distance(a, b):
    """|a - b| in float32 units in the last place (ordered-integer distance;
    +0 and -0 are 0 apart)."""
    ia = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    ib = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return np.abs(ia - ib)


def assert_float_output_within_1ulp(cams_a, pts_a, cams_b, pts_b, what=""):
    """Every entry of the write-back of solution a is identical to, or 1 ulp
    from, solution b's.  Returns {field: (entries, entries at 1 ulp)}."""
    fa = float_write_back(cams_a, pts_a)
    fb = float_write_back(cams_b, pts_b)
    stats = {}
    for name, x, y in zip(("R", "t", "pose", "points"), fa, fb):
        d = ulp_distance(x, y)
        stats[name] = (int(d.size), int((d == 1).sum()))
        assert d.size == 0 or d.max() <= 1, (f"{what} {name}: {int((d > 1).sum())} of {d.size} entries more than "
                                            f"1 ulp apart (max {int(d.max())})")
    print(f"float write-back {what}: entries / at 1 ulp {stats}")
    return stats
