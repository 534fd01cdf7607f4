"""Timeline of the last eigh in a rocprofv3 kernel trace (scripts/gpu_dc_wave.sh writes one):
every kernel from the last sytrd_ll_kernel start to the end of the call, with its start
relative to the reduction's end and its duration (us). python scripts/eigh_timeline.py <db>."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = list(c.execute("select name,start,end from kernels order by start"))
i = max(k for k, r in enumerate(rows) if "sytrd_ll_kernel" in r[0])
t0 = rows[i][2]
end = rows[i][2]
for name, st, en in rows[i:]:
    if st - end > 2_000_000:  # the next call starts after a gap (the bench's host work)
        break
    end = max(end, en)
    short = name.replace("(anonymous namespace)::", "").removeprefix("void ").split("(")[0].split("::")[-1][:60]
    print(f"{(st - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f}  {short}")
print(f"reduction end -> last kernel end: {(end - t0) / 1e3:.1f} us")
