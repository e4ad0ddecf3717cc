"""Average each PMC counter per kernel over dispatches from rocprofv3 csv dirs."""
import csv
import glob
import sys
from collections import defaultdict

def short(n):
    n = n.split("(")[0]
    return n.split("::")[-1]

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row.get("Kernel_Name", row.get("Kernel-Name", "?")))
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
want = sys.argv[2:] if False else None
for k in sorted(acc):
    if not k.startswith("k_"):
        continue
    vals = {c: sum(v) / len(v) for c, v in acc[k].items()}
    print(k, " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))
