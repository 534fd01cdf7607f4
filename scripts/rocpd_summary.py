#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (``*_results.db``) into top-kernel stats.

python scripts/rocpd_summary.py gpurun_out/x/prof/run_results.db [--out profiles/x/kernels.json] [--top 25]
"""
import argparse
import glob
import json
import os
import sqlite3


def summarize(db: str, top: int = 25) -> dict:
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
                          "max(vgpr_count), max(accum_vgpr_count), max(lds_size), max(grid_x), max(workgroup_x) "
                          "from kernels group by name order by sum(duration) desc"))
    total = sum(r[2] for r in rows) or 1
    out = []
    for r in rows[:top]:
        out.append({"kernel": r[0][:160], "calls": r[1], "total_ms": round(r[2] / 1e6, 4),
                    "avg_us": round(r[3] / 1e3, 3), "min_us": round(r[4] / 1e3, 3), "max_us": round(r[5] / 1e3, 3),
                    "pct": round(100.0 * r[2] / total, 2), "vgpr": r[6], "agpr": r[7], "lds": r[8],
                    "grid_x": r[9], "wg_x": r[10]})
    span = list(c.execute("select min(start), max(end) from kernels"))[0]
    return {"db": os.path.basename(db), "kernel_time_ms": round(total / 1e6, 3),
            "trace_span_ms": round((span[1] - span[0]) / 1e6, 3) if span[0] else None, "top": out}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db", nargs="+")
    ap.add_argument("--out", default="")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    dbs = [d for pat in a.db for d in (glob.glob(pat) or [pat])]
    res = [summarize(d, a.top) for d in dbs]
    txt = json.dumps(res if len(res) > 1 else res[0], indent=1)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    for r in res:
        print(f"{r['db']}: kernels {r['kernel_time_ms']} ms over {r['trace_span_ms']} ms span")
        for k in r["top"][:12]:
            print(f"  {k['pct']:6.2f}%  {k['total_ms']:10.3f} ms  {k['calls']:6d}x  {k['avg_us']:10.2f} us  {k['kernel'][:90]}")


if __name__ == "__main__":
    main()
