"""Summarise a rocprofv3 --stats kernel CSV: top kernels, per-step ms, grouped by category."""
import csv
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_classes import classify as cat  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
cats = {}


print(f"total GPU {tot / 1e6:.1f} ms over {steps:g} steps = {tot / 1e6 / steps:.1f} ms/step")
for r in rows:
    c = cat(r["Name"])
    cats[c] = cats.get(c, 0.0) + float(r["TotalDurationNs"])
for c, v in sorted(cats.items(), key=lambda x: -x[1]):
    print(f"  {c:40s} {v / 1e6 / steps:8.2f} ms/step {100 * v / tot:5.1f}%")
print("top kernels:")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    n = re.sub(r"\((?!anonymous).*", "", r["Name"])[:90]
    print(f"  {float(r['TotalDurationNs']) / 1e6 / steps:8.2f} ms/step {float(r['Percentage']):5.1f}% calls={r['Calls']:>5} {n}")
