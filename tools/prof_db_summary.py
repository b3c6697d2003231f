"""Top kernels of a rocprofv3 SQLite results database (the default output format):
python tools/prof_db_summary.py gpurun_out/prof/run_results.db [steps] [top]"""
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_classes import classify  # noqa: E402

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
c = sqlite3.connect(path)
rows = c.execute("select name, count(*), sum(duration) from kernels group by name order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"total GPU {tot / 1e6:.1f} ms over {steps:g} steps = {tot / 1e6 / steps:.2f} ms/step")
cats = {}
for name, cnt, d in rows:
    cats[classify(name)] = cats.get(classify(name), 0.0) + d
for c, d in sorted(cats.items(), key=lambda kv: -kv[1]):
    print(f"  {c:42s} {d / 1e6 / steps:8.2f} ms/step {100 * d / tot:5.1f}%")
print("top kernels:")
for name, cnt, d in rows[:top]:
    print(f"{d / 1e6 / steps:9.3f} ms/step {100 * d / tot:5.1f}%  calls/step {cnt / steps:7.1f}  {name[:110]}")
