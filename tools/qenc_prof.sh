#!/bin/bash
# rocprofv3 kernel stats of the query tower (bf16 BERT-base, 128 x 32 tokens, eager + graph)
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_qenc -o run --output-format csv -- \
  python3 -c "import sys, json, torch; sys.path.insert(0, '$R'); import bench_legs as bench_encode; print(json.dumps(bench_encode.run_query_encode(torch.device('cuda', 0))))" \
  > $R/gpurun_out/prof_qenc.log 2>&1
rc=$?
tail -1 $R/gpurun_out/prof_qenc.log
python3 - <<PY
import csv, glob
f = glob.glob("$R/gpurun_out/prof_qenc/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{float(r["TotalDurationNs"])/tot*100:5.1f}%  calls={r["Calls"]:>5s} avg={float(r["AverageNs"])/1e3:8.1f}us  {r["Name"][:100]}')
PY
exit $rc
