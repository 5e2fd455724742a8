#!/usr/bin/env python3
"""Kernel statistics (rocprofv3 --stats layout) from a rocprofv3 rocpd SQLite database.

usage: rocpd_stats.py RUN_results.db OUT.csv
Columns as rocprofv3's kernel_stats.csv: Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs, StdDev (durations from the `kernels` view, end - start of each dispatch)."""
import csv
import math
import sqlite3
import sys


def main():
    db, out = sys.argv[1:3]
    c = sqlite3.connect(db)
    rows = {}
    for name, start, end in c.execute("select name, start, end from kernels"):
        rows.setdefault(name, []).append(end - start)
    total = sum(sum(v) for v in rows.values())
    table = []
    for name, d in rows.items():
        n = len(d)
        mean = sum(d) / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in d) / n)
        table.append((name, n, sum(d), mean, 100.0 * sum(d) / total, min(d), max(d), sd))
    table.sort(key=lambda r: -r[2])
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for r in table:
            w.writerow([r[0], r[1], r[2], round(r[3], 3), round(r[4], 4), r[5], r[6], round(r[7], 3)])


if __name__ == "__main__":
    main()
