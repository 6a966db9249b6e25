"""Summarise a rocprofv3 SQLite kernel trace: top kernels and the per-call timeline gaps."""
import sqlite3
import sys

import numpy as np

db = sqlite3.connect(sys.argv[1])
rows = list(db.execute("select name,start,end from kernels order by start"))
print(f"{len(rows)} dispatches, span {(rows[-1][2] - rows[0][1]) / 1e6:.2f} ms")
for r in db.execute("select name,total_calls,total_duration,average,percentage from top_kernels limit 25"):
    # the rocpd top_kernels view reports durations in microseconds
    print(f"{r[0][:70]:70s} {r[1]:6d} total {r[2] / 1e3:9.2f}ms avg {r[3]:8.2f}us {r[4]:5.1f}%")
if len(sys.argv) > 2:
    n = int(sys.argv[2])
    t0, prev = rows[-n][1], None
    for name, s, e in rows[-n:]:
        gap = (s - prev) / 1e3 if prev else 0.0
        print(f"{(s - t0) / 1e3:9.1f} gap {gap:7.1f} dur {(e - s) / 1e3:7.1f} {name[:60]}")
        prev = e
