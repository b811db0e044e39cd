"""Kernel stats CSV (the columns of rocprofv3 --stats' kernel_stats.csv) from a rocprofv3 rocpd SQLite database.
    python scripts/rocpd_stats.py <run_results.db> <out.csv>"""
import csv
import sqlite3
import sys
from collections import defaultdict

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
d = defaultdict(list)
for n, s, e in rows:
    d[n].append(e - s)
tot = sum(sum(v) for v in d.values())
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for n, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        m = sum(v) / len(v)
        sd = (sum((x - m) ** 2 for x in v) / len(v)) ** 0.5
        w.writerow([n, len(v), sum(v), m, 100.0 * sum(v) / tot, min(v), max(v), sd])
print(out, len(d), "kernels")
