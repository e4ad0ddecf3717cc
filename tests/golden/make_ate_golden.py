"""Generate tests/golden/ate.json by running the reference's own ATE tools
(ba_project/src/metrics/evaluate_ate_scale.py + associate.py) on synthetic
TUM trajectories.  Runs only in the build container (needs /root/reference);
the fixture holds inputs (trajectory text) and outputs (numbers), no code.

    python tests/golden/make_ate_golden.py
"""
import contextlib
import io
import json
import os
import sys
import tempfile

import numpy as np

REF = "/root/reference/ba_project/src/metrics"


def traj_text(stamps, xyz, quat):
    return "".join(f"{s:.6f} {x:.6f} {y:.6f} {z:.6f} {a:.6f} {b:.6f} {c:.6f} {d:.6f}\n"
                   for s, (x, y, z), (a, b, c, d) in zip(stamps, xyz, quat))


def rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def case(rng, n, scale, noise, offset, jitter, drop, max_difference, planar=False):
    stamps = 1305031102.0 + np.arange(n) * 0.0333 + rng.uniform(-0.002, 0.002, n)
    tt = np.linspace(0, 2 * np.pi, n)
    gt = np.stack([np.cos(tt) * 1.5, np.sin(2 * tt) * 0.7, np.zeros(n) if planar else 0.2 * tt], 1) + rng.normal(0, 0.01, (n, 3))
    R, t = rot(rng), rng.normal(size=3)
    est = (gt - t) @ R / scale + rng.normal(0, noise, (n, 3))      # est = R^T (gt - t) / scale
    est_stamps = stamps - offset + rng.uniform(-jitter, jitter, n)
    keep = rng.uniform(size=n) > drop
    quat = np.tile([0.0, 0.0, 0.0, 1.0], (n, 1))
    return dict(gt=traj_text(stamps, gt, quat), est=traj_text(est_stamps[keep], est[keep], quat[keep]),
                offset=offset, scale=1.0, max_difference=max_difference)


def main():
    sys.path.insert(0, REF)
    import associate  # noqa: E402  (the reference's module)
    import evaluate_ate_scale as ev  # noqa: E402
    rng = np.random.default_rng(0xA7E)
    cases = [case(rng, 120, 0.5, 0.002, 0.0, 0.004, 0.0, 0.02),
             case(rng, 200, 3.7, 0.01, 0.5, 0.008, 0.15, 0.02),
             case(rng, 60, 1.0, 0.0, 0.0, 0.0, 0.1, 0.02, planar=True),
             case(rng, 90, 0.02, 0.0005, -0.25, 0.015, 0.3, 0.01)]
    out = []
    with tempfile.TemporaryDirectory() as d:
        for c in cases:
            g, e = os.path.join(d, "gt.txt"), os.path.join(d, "est.txt")
            open(g, "w").write(c["gt"])
            open(e, "w").write(c["est"])
            first, second = associate.read_file_list(g), associate.read_file_list(e)
            matches = associate.associate(first, second, float(c["offset"]), float(c["max_difference"]))
            fx = np.matrix([[float(v) for v in first[a][0:3]] for a, b in matches]).transpose()
            sx = np.matrix([[float(v) * c["scale"] for v in second[b][0:3]] for a, b in matches]).transpose()
            with contextlib.redirect_stdout(io.StringIO()):
                R, T, err, s = ev.align(sx, fx)
            err = np.asarray(err).reshape(-1)
            c = dict(c, expected=dict(pairs=len(matches), matches=[[a, b] for a, b in matches],
                                      rmse=float(np.sqrt(np.dot(err, err) / len(err))), mean=float(np.mean(err)),
                                      median=float(np.median(err)), std=float(np.std(err)), min=float(np.min(err)),
                                      max=float(np.max(err)), scale=float(s), rot=np.asarray(R).tolist(),
                                      trans=np.asarray(T).reshape(-1).tolist()))
            out.append(c)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ate.json")
    with open(path, "w") as f:
        json.dump(dict(source="ba_project/src/metrics/evaluate_ate_scale.py (align) + associate.py "
                              "(read_file_list, associate), run in the build container", cases=out), f)
    print(f"wrote {path}: {len(out)} cases")


if __name__ == "__main__":
    main()
