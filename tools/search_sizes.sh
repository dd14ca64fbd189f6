#!/bin/bash
# search bench at N=1 size and at the N=8 shard size (1.25M rows)
cd "$(dirname "$0")/.."
for n in ${SIZES:-10000000 1250000}; do
  timeout -k 10 300 python bench.py --n-corpus $n --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_n$n.log 2>&1 || exit $?
  grep '^{' gpurun_out/bench_n$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n', $n, d['value'], 'q/s', d['ms_per_step'], 'ms/step', d['roofline']['achieved'], 'GB/s scan', d['roofline']['avg_launch_ms'], 'ms')"
done
