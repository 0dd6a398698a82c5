#!/usr/bin/env python3
"""Per-kernel summary (calls, average / total ms) of a rocprofv3 --kernel-trace run saved in
its default rocpd SQLite format — the same numbers `--stats` prints, as CSV.
usage: scripts/rocpd_summary.py <results.db> [out.csv]"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, count(*), avg(duration), sum(duration), min(duration), max(duration) "
                  "from kernels group by name order by sum(duration) desc").fetchall()
out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
w = csv.writer(out)
w.writerow(["Name", "Calls", "AverageMs", "TotalMs", "MinMs", "MaxMs"])
for name, n, avg, tot, mn, mx in rows:
    w.writerow([name, n, f"{avg / 1e6:.4f}", f"{tot / 1e6:.3f}", f"{mn / 1e6:.4f}", f"{mx / 1e6:.4f}"])
