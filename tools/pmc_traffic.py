#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py into the HBM
traffic per launch of the dominant scan kernel (MI355X_MICROARCH.md, HBM:
FETCH_SIZE counts half the bytes of wide streaming reads on gfx950 -> x2;
WRITE_SIZE exact).  Writes profiles/<tag>_pmc_traffic.json, which bench.py
reports as roofline.traffic when its configuration matches.

usage: pmc_traffic.py <fetch_dir> <write_dir> <out.json> --n-corpus N --world W --qb Q --k K --dim D
"""
import argparse
import collections
import csv
import glob
import json


def per_kernel(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter and "drt::" in r["Kernel_Name"]:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--n-corpus", type=int, required=True)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--qb", type=int, default=128)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--launch-queries", type=int, default=0, help="a grouped launch: queries per filter launch")
    ap.add_argument("--launch-rows", type=int, default=0, help="a grouped launch: rows per filter launch")
    a = ap.parse_args()
    fetch = per_kernel(a.fetch_dir, "FETCH_SIZE")
    write = per_kernel(a.write_dir, "WRITE_SIZE")
    kernels = {}
    for name, v in fetch.items():
        w = write.get(name, [0.0])
        fkb = sorted(v)[len(v) // 2]
        wkb = sorted(w)[len(w) // 2]
        kernels[name] = {"launches": len(v), "fetch_size_kb_median": fkb, "write_size_kb_median": wkb,
                         "hbm_bytes_per_launch": 2 * fkb * 1024 + wkb * 1024}
    # the dominant kernel = the filter scan (the bench's roofline kernel; not row_stats, which reads the
    # corpus once per index and moves as many bytes in its single launch), else the largest mover
    scans = [k for k in kernels if "ip_scan16r_kernel" in k or "ip_scan32r_kernel" in k]
    scan = max(scans or kernels, key=lambda k: kernels[k]["hbm_bytes_per_launch"])
    cfg = {"n_corpus": a.n_corpus, "world": a.world, "qb": a.qb, "k": a.k, "dim": a.dim}
    if a.launch_queries:
        cfg.update(launch_queries=a.launch_queries, launch_rows=a.launch_rows)
    out = {"config": cfg,
           "dominant_kernel": scan, "traffic_bytes_per_launch": kernels[scan]["hbm_bytes_per_launch"],
           "correction": "HBM bytes = 2 x FETCH_SIZE (gfx950 wide-read tally) + WRITE_SIZE, KB = 1024 B",
           "kernels": kernels}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({"dominant_kernel": scan, "traffic_bytes_per_launch": out["traffic_bytes_per_launch"]}))


if __name__ == "__main__":
    main()
