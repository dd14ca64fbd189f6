"""Summarise tools/pmc_encode.sh: per kernel family, average duration, MFMA utilisation
(SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)) and effective clock
(GRBM_GUI_ACTIVE / 8 / duration)."""
import collections
import csv
import glob
import json
import sys


def main(d):
    f = glob.glob(d + "/**/run_counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(dict)
    for row in csv.DictReader(open(f)):
        key = (row["Dispatch_Id"], row["Kernel_Name"])
        per[key][row["Counter_Name"]] = float(row["Counter_Value"])
        for c in ("Start_Timestamp", "End_Timestamp"):
            if c in row:
                per[key][c] = int(row[c])
    trace = glob.glob(d + "/**/run_kernel_trace.csv", recursive=True)
    dur = {}
    if trace:
        for row in csv.DictReader(open(trace[0])):
            dur[row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    fam = collections.defaultdict(list)
    for (disp, name), c in per.items():
        if "drt::" not in name:
            continue
        t = dur.get(disp)
        if t is None and "End_Timestamp" in c:
            t = (c["End_Timestamp"] - c["Start_Timestamp"]) * 1e-9
        fam[name.split("(")[0][:80]].append((c, t))
    out = {}
    for name, rows in fam.items():
        g = sum(r[0].get("GRBM_GUI_ACTIVE", 0) for r in rows) / len(rows)
        m = sum(r[0].get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for r in rows) / len(rows)
        ts = [r[1] for r in rows if r[1]]
        t = sum(ts) / len(ts) if ts else None
        out[name] = {"launches": len(rows), "avg_us": round(t * 1e6, 1) if t else None,
                     "mfma_util": round(m / (1024 * g / 8), 4) if g else None,
                     "clock_ghz": round(g / 8 / t / 1e9, 3) if (g and t) else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
