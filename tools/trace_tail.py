#!/usr/bin/env python3
"""Decompose the tail of a rocprofv3 kernel trace: per-kernel busy time and the idle gaps
between consecutive kernels over the last N launches (the timed region of a tool run).

usage: python tools/trace_tail.py <rocprof output dir> [--last N] [--show M] [--match SUBSTR]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=400)
    ap.add_argument("--show", type=int, default=30)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    files = glob.glob(f"{args.dir}/**/*kernel_trace.csv", recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tail = rows[-args.last:]
    busy = collections.defaultdict(lambda: [0, 0.0])
    gaps = 0.0
    prev_end = None
    for r in tail:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0][:80]
        busy[name][0] += 1
        busy[name][1] += (e - s) / 1e3
        if prev_end is not None and s > prev_end:
            gaps += (s - prev_end) / 1e3
        prev_end = max(prev_end or e, e)
    span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
    print(f"last {len(tail)} kernels span {span:.1f} us; idle gaps {gaps:.1f} us ({gaps / span:.3f})")
    for name, (n, t) in sorted(busy.items(), key=lambda kv: -kv[1][1]):
        print(f"  {t:10.1f} us  {n:5d} x {t / n:8.2f} us  {name}")
    t0 = int(tail[-args.show]["Start_Timestamp"])
    for r in tail[-args.show:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f}us grid={r.get('Grid_Size_X', r.get('Grid_Size', '?')):>8s}"
              f" {r['Kernel_Name'][:90]}")
    if args.json:
        with open(args.json, "w") as fh:
            json.dump({"span_us": span, "gaps_us": gaps, "kernels": {k: {"n": v[0], "us": v[1]} for k, v in busy.items()}},
                      fh, indent=1)


if __name__ == "__main__":
    main()
