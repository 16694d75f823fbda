"""List full kernel names, grid sizes and mean durations from a rocprofv3 kernel-trace DB, for the
kernels whose shortened name matches a pattern: python bench/kernel_names.py DB PATTERN"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else ""
rows = c.execute("select name, grid_x, count(*), avg(duration) from kernels group by name, grid_x "
                 "order by count(*) * avg(duration) desc").fetchall()
for name, gx, n, d in rows:
    if pat in name:
        print(f"{n:6d} calls  {d / 1e3:9.1f} us  grid_x {gx:10d}  {name[:400]}")
