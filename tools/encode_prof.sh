#!/bin/bash
# rocprofv3 kernel stats of the encode leg (bf16 BERT-base, 512 x 128 tokens)
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_enc -o run --output-format csv -- \
  python3 -c "import sys, json, torch; sys.path.insert(0, '$R'); import bench_legs as bench_encode; print(json.dumps(bench_encode.run(torch.device('cuda', 0))))" \
  > $R/gpurun_out/prof_enc.log 2>&1
rc=$?
tail -2 $R/gpurun_out/prof_enc.log
python3 - <<PY
import csv, glob
f = glob.glob("$R/gpurun_out/prof_enc/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["TotalDurationNs"])/tot*100:5.1f}%  calls={r["Calls"]:>5s} avg={float(r["AverageNs"])/1e3:8.1f}us  {r["Name"][:110]}')
PY
exit $rc
