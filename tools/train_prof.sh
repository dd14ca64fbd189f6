#!/bin/bash
# rocprofv3 kernel stats of the C3 training step leg (HIP tower + HF fp32 reference)
#   LEG_ARGS='bq=128, n=8, p_len=156' profiles the recipe shape instead; TAG names the output dir
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train${TAG:-} -o run --output-format csv -- \
  python3 -c "import sys, json, torch; sys.path.insert(0, '$R'); import bench_legs as bench_encode; print(json.dumps(bench_encode.run_train_step(torch.device('cuda', 0), ${LEG_ARGS:-})))" \
  > $R/gpurun_out/prof_train${TAG:-}.log 2>&1
rc=$?
tail -1 $R/gpurun_out/prof_train${TAG:-}.log
python3 - <<PY
import csv, glob
f = glob.glob("$R/gpurun_out/prof_train${TAG:-}/**/run_kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "drt::" in r["Name"] or "rocclr" in r["Name"] or "at::" in r["Name"]]
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("drt + torch-elementwise total ms (4 steps):", round(tot / 1e6, 1))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:28]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.1f} ms calls={r["Calls"]:>5s} avg={float(r["AverageNs"])/1e3:8.1f}us  {r["Name"][:95]}')
PY
exit $rc
