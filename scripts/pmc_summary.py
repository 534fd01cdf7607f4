#!/usr/bin/env python3
"""Shrink a rocprofv3 output directory to a small summary (run on the GPU box).

For every ``*counter_collection.csv`` under DIR: sum each counter per kernel name over its
dispatches (kernels whose name matches --match); for every ``*kernel_stats.csv`` keep the
top rows. Writes DIR/summary.json and deletes the large per-dispatch CSV / trace files so
the directory fits gpurun's copy-back limit.

python scripts/pmc_summary.py DIR [--match REGEX] [--keep]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default=".")
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    rx = re.compile(a.match)
    out = {"counters": {}, "kernel_stats": {}}
    for fn in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        agg = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        with open(fn) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "?")
                if not rx.search(k):
                    continue
                agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row.get("Dispatch_Id", ""))
        out["counters"][os.path.relpath(fn, a.dir)] = {
            k[:160]: {"dispatches": len(disp[k]), **{c: v for c, v in sorted(cs.items())}} for k, cs in agg.items()}
    for fn in glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True):
        with open(fn) as f:
            rows = list(csv.DictReader(f))
        out["kernel_stats"][os.path.relpath(fn, a.dir)] = [
            {"name": r["Name"][:160], "calls": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6,
             "avg_us": float(r["AverageNs"]) / 1e3, "pct": float(r["Percentage"]),
             "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3} for r in rows[:25]]
    with open(os.path.join(a.dir, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    if not a.keep:
        for pat in ("*counter_collection.csv", "*kernel_trace.csv", "*.db", "*agent_info.csv", "*.pftrace"):
            for fn in glob.glob(os.path.join(a.dir, "**", pat), recursive=True):
                os.remove(fn)


if __name__ == "__main__":
    main()
