"""Per-kernel totals over the LAST `ms` milliseconds of a rocprofv3 kernel trace (the timed
steps), so warm-up / autotuning kernels are excluded. usage: trace_window.py trace.csv ms steps"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_classes import classify  # noqa: E402

path, ms, steps = sys.argv[1], float(sys.argv[2]), float(sys.argv[3])
rows = list(csv.DictReader(open(path)))
end = max(int(r["End_Timestamp"]) for r in rows)
start = end - ms * 1e6
agg, busy = {}, 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < start:
        continue
    d = e - s
    busy += d
    a = agg.setdefault(r["Kernel_Name"], [0, 0])
    a[0] += d
    a[1] += 1
print(f"window {ms} ms, kernel busy {busy / 1e6:.2f} ms = {busy / 1e6 / steps:.2f} ms/step")
cats = {}
for n, (d, c) in agg.items():
    k = classify(n)
    cats[k] = cats.get(k, 0) + d
for k, v in sorted(cats.items(), key=lambda x: -x[1]):
    print(f"  {k:40s} {v / 1e6 / steps:8.2f} ms/step {100 * v / busy:5.1f}%")
for n, (d, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:30]:
    print(f"{d / 1e6 / steps:8.3f} ms/step {c / steps:6.1f}/step  {n[:120]}")
