"""Per-launch-shape durations of the filter scan from a rocprofv3 kernel trace (csv): every
ip_scan32r_kernel launch grouped by its grid (the launch shape), in issue order, with the per-shape
average -- the figure bench.py's roofline.per_shape reports from HIP events.
usage: python tools/scan_shape_stats.py <run_kernel_trace.csv> <out.json>"""
import csv
import json
import sys


def main(path, out):
    rows = [r for r in csv.DictReader(open(path)) if "ip_scan32r_kernel" in r.get("Kernel_Name", "")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gk = [k for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z", "Grid_Size") if k in (rows[0] if rows else {})]
    shapes = {}
    seq = []
    for r in rows:
        g = "x".join(r[k] for k in gk)
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        shapes.setdefault(g, []).append(us)
        seq.append([g, round(us, 1)])
    res = {"kernel": "ip_scan32r_kernel<768>", "launches": len(rows), "grid_fields": gk,
           "per_grid": {g: {"launches": len(v), "avg_us": round(sum(v) / len(v), 1),
                            "last8_avg_us": round(sum(v[-8:]) / len(v[-8:]), 1)} for g, v in shapes.items()},
           "sequence": seq}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["per_grid"]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
