"""Timeline of one k_chol_flow launch (the split Cholesky's flow form) from
tools/chol_bench_ft (built with -DBA_CHOL_FLOW_TRACE), which writes the task
list and each task's s_memrealtime stamps (start, after its waits, end; 100
MHz) to flow_trace.bin.

    python3 tools/flow_trace.py flow_trace.bin
"""
import struct
import sys

import numpy as np


def main():
    raw = open(sys.argv[1], "rb").read()
    nt = struct.unpack_from("<I", raw, 0)[0]
    tasks = np.frombuffer(raw, dtype=np.int32, count=4 * nt, offset=4).reshape(nt, 4)
    st = np.frombuffer(raw, dtype=np.uint64, count=4 * nt, offset=4 + 16 * nt).reshape(nt, 4).astype(np.int64)
    t0 = st[:, 0].min()
    s, w, e = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0, (st[:, 2] - t0) / 100.0   # us
    crit = (tasks[:, 0] >> 21) & 1 == 1
    col = ((tasks[:, 0] >> 20) & 1 == 1) & ~crit
    ranks = np.where(crit, 0, tasks[:, 3] - tasks[:, 2])
    total = e.max()
    print(f"{nt} tasks, {total:.1f} us from the first start to the last end")
    busy = (e - w)[~crit].sum()
    wait = (w - s)[~crit].sum()
    print(f"tile tasks: run {busy / 1e3:.1f} ms-slots, waiting {wait / 1e3:.1f} ms-slots; "
          f"over 512 slots x {total:.0f} us = {512 * total / 1e3:.1f} ms-slots -> run {busy / (512 * total):.2f}, "
          f"wait {wait / (512 * total):.2f}")
    pr = ranks[~crit & (ranks > 0)]
    dur = (e - w)[~crit & (ranks > 0)]
    for r in sorted(set(pr.tolist()))[:8]:
        m = pr == r
        print(f"  rank {r:2d} x64: {m.sum():6d} tasks, run {np.median(dur[m]):6.1f} us median, "
              f"{np.percentile(dur[m], 90):6.1f} p90")
    off = 4 + 16 * nt + 32 * nt
    if len(raw) > off:
        nc = struct.unpack_from("<I", raw, off)[0]
        ch = np.frombuffer(raw, dtype=np.uint64, count=6 * nc, offset=off + 4).reshape(nc, 6).astype(np.int64)
        ph = (ch[:, [2, 3, 4, 1]] - ch[:, [0, 2, 3, 4]]) / 100.0
        print("chain phases (us, mean): tile loads + puts %.1f  panel row P + A_dd put %.1f  C col0 + factor %.1f"
              "  V out + publish %.1f" % tuple(ph.mean(axis=0)))
        ready, done = (ch[:, 0] - t0) / 100.0, (ch[:, 1] - t0) / 100.0
        step = done - ready
        waitk = ready[1:] - done[:-1]
        print(f"chain workgroup: {nc} steps, work {step.sum():.0f} us ({step.mean():.1f} mean), waiting for inputs "
              f"{waitk.sum():.0f} us ({np.median(waitk):.1f} median); last V at {done[-1]:.0f} us")
        for k in list(range(0, nc, max(1, nc // 12))) + [nc - 1]:
            wk = ready[k] - done[k - 1] if k else ready[k]
            print(f"  k={k:3d}: inputs ready {ready[k]:8.1f} (+{wk:6.1f})  V published {done[k]:8.1f}  ({step[k]:5.1f})")
    ci = np.nonzero(crit)[0]
    ks = tasks[ci, 1]
    order = np.argsort(ks)
    ci = ci[order]
    print("critical tasks (us): step, start, waited, ran, interval since the previous critical's end")
    prev_end = 0.0
    gaps = []
    runs = []
    for j, i in enumerate(ci):
        k = tasks[i, 1]
        gap = s[i] - prev_end if j else 0.0
        runs.append(e[i] - w[i])
        if j:
            gaps.append(w[i] - prev_end)
        if j < 6 or j % 10 == 0 or j + 3 > len(ci):
            print(f"  k={k:3d} start {s[i]:8.1f} waited {w[i] - s[i]:6.1f} ran {e[i] - w[i]:5.1f} "
                  f"(ready {w[i] - prev_end:6.1f} after the previous critical ended)")
        prev_end = e[i]
    print(f"critical: ran {np.sum(runs):.0f} us total ({np.mean(runs):.1f} mean); ready-after-previous "
          f"{np.sum(gaps):.0f} us total ({np.mean(gaps):.1f} mean, {np.median(gaps):.1f} median)")
    # column tasks of each step: their last end relative to the step's critical end
    lag = []
    for i in ci:
        k = tasks[i, 1]
        m = col & (tasks[:, 1] == k + 1)
        if m.any():
            lag.append(e[m].max() - e[i])
    if lag:
        print(f"column tasks: last one ends {np.mean(lag):.1f} us (mean) after their step's critical")
    # occupancy over time
    grid = np.linspace(0, total, 21)
    occ = [(np.sum((s <= x) & (e > x)), np.sum((w <= x) & (e > x))) for x in grid[1:-1]]
    print("resident / running tasks at 5 % marks:", " ".join(f"{a}/{b}" for a, b in occ))


if __name__ == "__main__":
    main()
