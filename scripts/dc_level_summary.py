"""Per-level durations of the D&C kernels (csrc/tridiag_dc.hip) in the last eigh of a rocprofv3
kernel trace: python scripts/dc_level_summary.py <run_results.db>. The last eigh is the last run
of dc_ kernels without a gap of more than 1 ms (the reduction separates two calls)."""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = list(c.execute("select name,start,end,grid_x,grid_y,workgroup_x from kernels "
                      "where name like '%anonymous namespace)::dc_%' order by start"))
i = len(rows) - 1
while i > 0 and rows[i][1] - rows[i - 1][2] < 1_000_000:
    i -= 1
last = rows[i:]
tot = collections.Counter()
for r in last:
    tot[r[0].split('::')[1][:18]] += (r[2] - r[1]) / 1e3
print({k: round(v, 1) for k, v in tot.items()}, round(sum(tot.values()), 1), 'span',
      round((last[-1][2] - last[0][1]) / 1e3, 1))
for r in last:
    print(r[0].split('::')[1][:18], round((r[2] - r[1]) / 1e3, 1), r[3], r[4])
