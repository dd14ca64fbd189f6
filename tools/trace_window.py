#!/usr/bin/env python3
"""Print the kernel-trace window around the first launch of a kernel whose name contains MATCH
(and whose grid is at least --min-grid): start offset, idle gap before, duration, grid, name.
usage: python tools/trace_window.py <rocprof dir> MATCH [--before 30] [--after 4] [--min-grid 0] [--nth 0]"""
from __future__ import annotations

import argparse
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("match")
    ap.add_argument("--before", type=int, default=30)
    ap.add_argument("--after", type=int, default=4)
    ap.add_argument("--min-grid", type=int, default=0)
    ap.add_argument("--nth", type=int, default=0)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    hits = [i for i, r in enumerate(rows)
            if a.match in r["Kernel_Name"] and int(r.get("Grid_Size_X", "0") or 0) >= a.min_grid]
    if len(hits) <= a.nth:
        print(f"no launch #{a.nth} of {a.match}")
        return
    i = hits[a.nth]
    lo = max(0, i - a.before)
    t0 = int(rows[lo]["Start_Timestamp"])
    prev = None
    for r in rows[lo: i + a.after + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(s - t0) / 1e3:10.1f} gap{gap:8.1f} {(e - s) / 1e3:9.1f}us grid={r.get('Grid_Size_X')} "
              f"{r['Kernel_Name'][:70]}")
        prev = e


if __name__ == "__main__":
    main()
