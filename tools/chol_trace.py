"""Per-step timeline of the split Cholesky from a rocprofv3 kernel trace of
tools/chol_bench_ns (its last streamed factorisation): for each block step,
the panel launch, the update launch and the gaps between them.

    python3 tools/chol_trace.py <dir containing *kernel_trace.csv>
"""
import csv
import glob
import os
import sys


def main():
    f = sorted(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    # the last streamed factorisation: the last k_chol_step (k = -1) before the
    # final k_back_flow, up to that back_flow
    ends = [i for i, n in enumerate(names) if "k_back_flow" in n]
    # the streamed runs come after the per-step runs: take the second-to-last
    # back_flow's preceding factor if the last one is the persistent form
    last_bf = ends[-1]
    first = max(i for i in range(last_bf) if "k_chol_step" in names[i] and "split" not in names[i])
    seq = rows[first:last_bf]
    t0 = int(seq[0]["Start_Timestamp"])
    steps = []
    i = 1
    while i + 1 < len(seq):
        p, u = seq[i], seq[i + 1]
        steps.append((int(p["Start_Timestamp"]), int(p["End_Timestamp"]), int(u["Start_Timestamp"]),
                      int(u["End_Timestamp"]), u.get("Grid_Size_X", u.get("Grid_Size", "?"))))
        i += 2
    tot = int(seq[-1]["End_Timestamp"]) - t0
    print(f"{os.path.basename(f)}: {len(steps)} steps, {tot / 1e3:.1f} us from diag 0 to the last update")
    sp = su = sg = 0
    prev_end = int(seq[0]["End_Timestamp"])
    for k, (ps, pe, us, ue, grid) in enumerate(steps):
        sp += pe - ps
        su += ue - us
        sg += (ps - prev_end) + (us - pe)
        if k < 12 or k % 8 == 0 or k + 3 > len(steps):
            print(f"step {k:3d}: gap {(ps - prev_end) / 1e3:5.1f}  panel {(pe - ps) / 1e3:5.1f}  gap {(us - pe) / 1e3:5.1f}"
                  f"  update {(ue - us) / 1e3:6.1f} us  (grid {grid})")
        prev_end = ue
    print(f"sums: panel {sp / 1e3:.1f}  update {su / 1e3:.1f}  gaps {sg / 1e3:.1f} us")


if __name__ == "__main__":
    main()
