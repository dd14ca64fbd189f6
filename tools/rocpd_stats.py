#!/usr/bin/env python3
"""Kernel stats (calls, average / total duration) from a rocprofv3 rocpd database (run_results.db), in
the column layout of rocprofv3's --stats kernel_stats.csv.  usage: tools/rocpd_stats.py <db> [out.csv]"""
import csv
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), "
                     f"max(end - start) from kernels group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    out = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
    out.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for n, calls, s, a, mn, mx in rows:
        out.writerow([n, calls, s, round(a, 1), round(100.0 * s / tot, 3), mn, mx])


if __name__ == "__main__":
    main()
