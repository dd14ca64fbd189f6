#!/bin/bash
# Perf probes: GEMM variants vs hipBLASLt; scan streaming ceiling.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 || exit $?
tail -1 gpurun_out/gemm_bench.log
for v in 0 1; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --scan-variant $v > gpurun_out/scanvar_$v.log 2>&1 || exit $?
  grep '^{' gpurun_out/scanvar_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('variant', $v, d['roofline']['achieved'], 'GB/s', d['roofline']['avg_launch_ms'], 'ms')"
done
