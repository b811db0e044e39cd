"""Kernel stats CSV (the columns of rocprofv3 --stats' kernel_stats.csv) from a rocprofv3 rocpd SQLite database, and
<out>_by_grid.csv with the same per (kernel, grid size): one row per layer of a kernel several layers share.
    python scripts/rocpd_stats.py <run_results.db> <out.csv>"""
import csv
import sqlite3
import sys
from collections import defaultdict

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
rows = c.execute(f"select {name_col}, start, end, grid_x, grid_y, grid_z from kernels").fetchall()
d = defaultdict(list)
dg = defaultdict(list)   # per (kernel, grid): one layer of a multi-layer kernel (e.g. g_a.2.dgrad vs g_a.4.dgrad)
for n, s, e, gx, gy, gz in rows:
    d[n].append(e - s)
    dg[(n, gx, gy, gz)].append(e - s)
tot = sum(sum(v) for v in d.values())
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for n, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        m = sum(v) / len(v)
        sd = (sum((x - m) ** 2 for x in v) / len(v)) ** 0.5
        w.writerow([n, len(v), sum(v), m, 100.0 * sum(v) / tot, min(v), max(v), sd])
with open(out[:-4] + "_by_grid.csv", "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Grid", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
    for (n, gx, gy, gz), v in sorted(dg.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([n, f"{gx}x{gy}x{gz}", len(v), sum(v), sum(v) / len(v), min(v), max(v)])
print(out, len(d), "kernels")
