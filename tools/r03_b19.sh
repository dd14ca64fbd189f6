#!/bin/bash
# Round 3 session B19: HEAD on MI355X -- GPU tests, smoke, bench, rocprof stats and the two PMC
# traffic passes (tools/r03_check.sh with PMC=1), then the bench's N > 1 code path rehearsed with
# two gloo ranks sharing the one GPU (ShardedFlatIP, grouped global-threshold protocol).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
TAG=${TAG:-r03zj}
PMC=1 TAG=$TAG STEPS=20 bash tools/r03_check.sh || exit $?
cd $R
DRT_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 6 --warmup 2 --n-corpus 2000000 \
  --no-cpu-baseline --no-encode > gpurun_out/${TAG}_gloo2.log 2>&1; rc=$?
echo "=== gloo2 rc=$rc"; tail -2 gpurun_out/${TAG}_gloo2.log
exit $rc
