#!/usr/bin/env python3
"""Kernel summary (name, calls, total/avg ns, %) from a rocprofv3 SQLite output
(rocpd `top_kernels` view), as CSV - for runs made without --output-format csv."""
import csv
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
cur = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for r in cur:
        w.writerow(r)
