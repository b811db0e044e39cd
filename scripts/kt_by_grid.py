"""Per-(kernel, grid) durations from a rocprofv3 --kernel-trace CSV (one row per layer of a kernel that several
layers share), so the raw trace need not leave the GPU box.
    python scripts/kt_by_grid.py <kernel_trace.csv> <out_by_grid.csv>"""
import csv
import sys
from collections import defaultdict

src, out = sys.argv[1], sys.argv[2]
d = defaultdict(list)
for r in csv.DictReader(open(src)):
    g = (r.get("Grid_Size") or "x".join(r.get(k, "") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z")))
    d[(r["Kernel_Name"], g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Grid", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
    for (n, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([n, g, len(v), sum(v), sum(v) / len(v), min(v), max(v)])
