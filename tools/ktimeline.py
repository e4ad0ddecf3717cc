"""Kernel timeline of one LM step from a rocprofv3 kernel trace: start / end
relative to the step's point-elimination kernel (us), with the queue."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_point_elim"
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i = idx[-2] if len(idx) > 1 else idx[-1]
t0 = int(rows[i]["Start_Timestamp"])
for r in rows[i:i + 14]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{r['Kernel_Name'][:44]:44s} q{r['Queue_Id']:>3s} start {s / 1000:8.1f} end {e / 1000:8.1f} dur {(e - s) / 1000:7.1f}")
