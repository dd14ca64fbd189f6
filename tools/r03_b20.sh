#!/bin/bash
# Round 3 session B20: PMC HBM-traffic passes of the headline search alone (the full bench under
# --pmc segfaulted inside the runtime during the encoder legs: profiles/r03zj_pmc_fetch_crash.log),
# then the C2 evaluate leg with the full-query-set warm-up, then the N > 1 bench path rehearsed
# with two gloo ranks sharing the one GPU.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${TAG:-r03zk}
cd /tmp
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_${TAG}_$C -o run \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-encode > $OUT/pmc_${TAG}_$C.log 2>&1
  rc=$?; echo "=== pmc $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 $R/tools/pmc_traffic.py $OUT/pmc_${TAG}_FETCH_SIZE $OUT/pmc_${TAG}_WRITE_SIZE $OUT/${TAG}_pmc_traffic.json --n-corpus 10000000 || exit 1
cd $R
timeout -k 10 300 python3 -u -c "
import json, torch, bench_legs
print(json.dumps(bench_legs.run_evaluate_c2(torch.device('cuda', 0))), flush=True)" > $OUT/${TAG}_evaluate_c2.log 2>&1; rc=$?
echo "=== c2 rc=$rc"; tail -1 $OUT/${TAG}_evaluate_c2.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
DRT_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 6 --warmup 2 --n-corpus 2000000 \
  --no-cpu-baseline --no-encode > $OUT/${TAG}_gloo2.log 2>&1; rc=$?
echo "=== gloo2 rc=$rc"; grep '^{' $OUT/${TAG}_gloo2.log | cut -c1-400
exit $rc
