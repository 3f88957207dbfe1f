"""Print consecutive runs of one kernel name from a rocprofv3 rocpd database (mean/min us per run)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name}, end-start from kernels order by start").fetchall()
runs = []
for n, d in rows:
    if runs and runs[-1][0] == n:
        runs[-1][1].append(d)
    else:
        runs.append([n, [d]])
for n, ds in runs:
    if len(ds) >= 5 or "advance" in n:
        print(f"{len(ds):4d} x {n[:60]:60s} mean {sum(ds) / len(ds) / 1e3:8.2f} us  min {min(ds) / 1e3:8.2f} us")
