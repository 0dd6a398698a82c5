#!/usr/bin/env python3
"""Print the kernel timeline (name, start offset, duration, grid) from a rocprofv3 SQLite
result (rocprofv3 --kernel-trace -d DIR -o run): scripts/kernel_timeline.py DB [LAST_N]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = db.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
t0 = rows[-last][1] if len(rows) >= last else rows[0][1]
for name, s, e, g, w in rows[-last:]:
    print(f"{(s - t0) / 1e6:9.3f} ms  {(e - s) / 1e6:8.3f} ms  grid {g // max(w, 1):>8} x {w:<5} {name[:90]}")
