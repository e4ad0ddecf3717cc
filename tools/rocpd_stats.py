"""Per-kernel stats (calls, average, total, share) from a rocprofv3 SQLite
output (rocpd_*.db), in the column layout of rocprofv3's kernel_stats.csv:
  python3 tools/rocpd_stats.py gpurun_out/prof/x_results.db [out.csv]"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("""select s.kernel_name, count(*), sum(d.end - d.start), min(d.end - d.start), max(d.end - d.start)
                     from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
                     group by s.kernel_name order by sum(d.end - d.start) desc""").fetchall()
tot = sum(r[2] for r in rows) or 1
out = [["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]]
for name, n, t, mn, mx in rows:
    out.append([name, n, t, round(t / n, 1), round(100.0 * t / tot, 2), mn, mx])
if len(sys.argv) > 2:
    with open(sys.argv[2], "w", newline="") as f:
        csv.writer(f).writerows(out)
for r in out[1:]:
    print(f"{r[0][:72]:72s} {r[1]:6d} {r[3] / 1e3:10.1f} us {r[4]:6.2f} %")
