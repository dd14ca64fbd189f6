#!/bin/bash
# rocprofv3 kernel stats of the rerank leg (bf16 BERT-base cross-encoder, 1000 pairs x 160 tokens)
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rr -o run --output-format csv -- \
  python3 -c "import sys, json, torch; sys.path.insert(0, '$R'); import bench_legs as b; print(json.dumps(b.run_rerank(torch.device('cuda', 0))))" \
  > $R/gpurun_out/prof_rr.log 2>&1
rc=$?
tail -1 $R/gpurun_out/prof_rr.log | cut -c1-300
f=$(find /tmp/prof_rr -name "run_kernel_stats.csv" | head -1)
cp $f $R/gpurun_out/rerank_kernel_stats.csv
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$R/gpurun_out/rerank_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["TotalDurationNs"])/tot*100:5.1f}%  calls={r["Calls"]:>5s} avg={float(r["AverageNs"])/1e3:8.1f}us  {r["Name"][:110]}')
PY
exit $rc
