"""Per-level durations of the D&C kernels (csrc/tridiag_dc.hip) in the last eigh of a rocprofv3
kernel trace: python scripts/dc_level_summary.py <run_results.db>."""
import sqlite3,sys,collections
c=sqlite3.connect(sys.argv[1])
rows=list(c.execute("select name,start,end,grid_x,grid_y,workgroup_x from kernels where name like '%anonymous namespace)::dc_%' order by start"))
last=rows[-60:]
tot=collections.Counter()
for r in last: tot[r[0].split('::')[1][:18]]+= (r[2]-r[1])/1e3
print({k:round(v,1) for k,v in tot.items()}, round(sum(tot.values()),1), 'span', round((last[-1][2]-last[0][1])/1e3,1))
for r in last[-18:]: print(r[0].split('::')[1][:18], round((r[2]-r[1])/1e3,1), r[3], r[4])
