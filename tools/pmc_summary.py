#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 PMC passes (tools/pmc_linearize.sh).

FETCH_SIZE and WRITE_SIZE come from separate passes (they do not fit one
pass on gfx950).  Both are reported by rocprofv3 in KiB per dispatch;
FETCH_SIZE is doubled per MI355X_MICROARCH.md (on gfx950 it reports half the
bytes of wide streaming reads).  Writes profiles/pmc_<config>.json, which
bench.py reads for roofline.traffic.

usage: tools/pmc_summary.py <pmc_FETCH_SIZE dir> <pmc_WRITE_SIZE dir> <out.json> [algorithmic_bytes]
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def per_kernel(d: Path, counter: str):
    vals = defaultdict(list)
    for f in d.rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter:
                    vals[row["Kernel_Name"]].append(float(row["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("algo", nargs="?", type=float, default=None)
    ap.add_argument("--sq", default=None, help="SQ pass dir: SQ_INSTS_VALU per launch joins the record")
    ap.add_argument("--n-obs", type=int, default=None, help="observations of the profiled problem (per rank)")
    a = ap.parse_args()
    fdir, wdir, out, algo = Path(a.fetch_dir), Path(a.write_dir), Path(a.out), a.algo
    fetch, nf = per_kernel(fdir, "FETCH_SIZE")
    write, nw = per_kernel(wdir, "WRITE_SIZE")
    valu = per_kernel(Path(a.sq), "SQ_INSTS_VALU")[0] if a.sq else {}
    res = {}
    for k in sorted(set(fetch) | set(write)):
        short = k.split("(")[0].replace("bahip::", "").replace("void ", "").split("<")[0].strip()
        if short.startswith("k_linearize"):   # the roofline kernel, whichever variant ran
            short = "k_linearize"
        fb = 2.0 * fetch.get(k, 0.0)
        wb = write.get(k, 0.0)
        res[short] = {"fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                      "hbm_bytes_per_launch": fb + wb, "dispatches": [nf.get(k, 0), nw.get(k, 0)]}
        if k in valu:   # (per_kernel scales by 1024 for the KiB counters: undo)
            res[short]["valu_insts_per_launch"] = valu[k] / 1024.0
    res["_note"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes of `bench.py --steps 3`; "
                    "FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md); KiB -> bytes")
    if a.n_obs:
        res["_problem"] = {"n_obs": a.n_obs}
    if algo and "k_linearize" in res:
        res["k_linearize"]["algorithmic_bytes"] = algo
        res["k_linearize"]["traffic_over_algorithmic"] = res["k_linearize"]["hbm_bytes_per_launch"] / algo
    out.write_text(json.dumps(res, indent=1))
    for k, v in res.items():
        if not k.startswith("_"):
            print(f"{k:32s} fetch {v['fetch_bytes_per_launch'] / 1e6:9.2f} MB  write {v['write_bytes_per_launch'] / 1e6:9.2f} MB")


if __name__ == "__main__":
    main()
