"""Summarise a rocprofv3 kernel_stats.csv: per-kernel calls, avg/total time."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else None
for r in rows:
    n = r['Name'].split('(')[0].replace('bahip::', '')
    tot = float(r['TotalDurationNs']) / 1e3
    extra = f" per_step_us={tot / steps:8.1f}" if steps else ""
    print(f"{n:30s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.2f} total_us={tot:10.1f} pct={float(r['Percentage']):6.2f}{extra}")
