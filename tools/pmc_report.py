"""Per-kernel averages of every PMC counter in one or more rocprofv3 --pmc runs (csv output):
kernel name -> {counter: mean value per dispatch, avg_us from the kernel trace}."""
import collections
import csv
import glob
import json
import sys


def main(dirs):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        f = glob.glob(d + "/**/run_counter_collection.csv", recursive=True)
        if not f:
            continue
        per = collections.defaultdict(dict)
        for row in csv.DictReader(open(f[0])):
            per[(row["Dispatch_Id"], row["Kernel_Name"].split("(")[0][:90])][row["Counter_Name"]] = \
                float(row["Counter_Value"])
        trace = glob.glob(d + "/**/run_kernel_trace.csv", recursive=True)
        dur = {}
        if trace:
            for row in csv.DictReader(open(trace[0])):
                dur[row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3
        for (disp, name), c in per.items():
            for k, v in c.items():
                out[name][k].append(v)
            if disp in dur:
                out[name]["avg_us"].append(dur[disp])
    res = {n: {k: round(sum(v) / len(v), 2) for k, v in c.items()} for n, c in out.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
