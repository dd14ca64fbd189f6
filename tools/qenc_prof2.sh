#!/bin/bash
# rocprofv3 kernel stats of the query tower per batch size (bf16 BERT-base, 32 tokens, eager, 20 forwards)
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
for B in 8 128; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_q$B -o run --output-format csv -- \
  python3 -c "import sys, json, torch; sys.path.insert(0, '$R'); import bench_legs as bench_encode; print(json.dumps(bench_encode.run_query_encode(torch.device('cuda', 0), batches=($B,), steps=20)))" \
  > $R/gpurun_out/prof_q$B.log 2>&1 || exit $?
tail -1 $R/gpurun_out/prof_q$B.log
python3 - <<PY
import csv, glob
f = glob.glob("$R/gpurun_out/prof_q$B/**/run_kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f))]
nfwd = 2 * (20 + 3)   # eager + graph, steps + warmup
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("batch $B: kernel time per forward %.1f us" % (tot / nfwd / 1e3))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["TotalDurationNs"])/nfwd/1e3:8.1f} us/fwd calls/fwd={int(r["Calls"])/nfwd:5.1f} avg={float(r["AverageNs"])/1e3:7.1f}us  {r["Name"][:90]}')
PY
done
