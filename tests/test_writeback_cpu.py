"""The float write-back comparison helper (tests/writeback.py) on known cases."""
import numpy as np

from writeback import float_write_back, ulp_distance


def test_ulp_distance_known_cases():
    one = np.float32(1.0)
    up = np.nextafter(one, np.float32(2.0))
    assert ulp_distance([one], [up])[0] == 1
    assert ulp_distance([np.float32(0.0)], [np.float32(-0.0)])[0] == 0
    tiny = np.nextafter(np.float32(0.0), np.float32(1.0))
    assert ulp_distance([tiny], [-tiny])[0] == 2            # across zero
    assert ulp_distance([-one], [-up])[0] == 1
    assert ulp_distance([np.float32(3.0)], [np.float32(3.0)])[0] == 0


def test_write_back_of_a_pose_inverts_it():
    rng = np.random.default_rng(1)
    cams = np.column_stack([rng.normal(0, 0.5, (20, 3)), rng.normal(0, 2, (20, 3))])
    R, t, pose, X = float_write_back(cams, rng.normal(size=(5, 3)))
    assert R.dtype == t.dtype == pose.dtype == X.dtype == np.float32
    E = np.zeros((20, 4, 4)); E[:, :3, :3] = R; E[:, :3, 3] = t; E[:, 3, 3] = 1
    np.testing.assert_allclose(pose.astype(np.float64) @ E, np.broadcast_to(np.eye(4), E.shape), atol=1e-5)
    # identical inputs -> identical write-back
    again = float_write_back(cams, X)
    assert all(np.array_equal(a, b) for a, b in zip((R, t, pose), again[:3]))
