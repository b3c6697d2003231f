"""Summarise a rocprofv3 --pmc SQLite database on the box (the raw database is too big to copy
back): the schema, then per kernel name the dispatch count, total duration and each counter's
sum.  python tools/pmc_db_dump.py DB [name-substring ...]"""
import sqlite3
import sys

db = sys.argv[1]
keys = sys.argv[2:]
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
print("tables:", tabs)
for t in tabs:
    if any(k in t.lower() for k in ("pmc", "counter", "kernel")):
        cols = [r[1] for r in c.execute(f"pragma table_info('{t}')")]
        print(f"  {t}: {cols}")
# kernels: durations
rows = c.execute("select name, count(*), sum(duration) from kernels group by name order by sum(duration) desc").fetchall()
for n, cnt, d in rows[:12]:
    if not keys or any(k in n for k in keys):
        print(f"KERNEL {cnt:6d} {d / 1e6:10.3f} ms  {n[:110]}")
# counters: try the common layouts
for t in tabs:
    cols = [r[1] for r in c.execute(f"pragma table_info('{t}')")]
    low = [x.lower() for x in cols]
    if "value" in low and any(x in low for x in ("counter_name", "name")) and t != "kernels":
        cn = cols[low.index("counter_name")] if "counter_name" in low else cols[low.index("name")]
        kid = next((cols[low.index(x)] for x in ("kernel_name", "kernel_id", "dispatch_id", "correlation_id") if x in low), None)
        print(f"counter table {t} via {cn}, key {kid}")
        try:
            q = f"select {kid}, {cn}, sum(value), count(*) from '{t}' group by {kid}, {cn}"
            for r in c.execute(q).fetchall()[:400]:
                print("  ", r)
        except Exception as e:  # noqa: BLE001
            print("  query failed:", e)
