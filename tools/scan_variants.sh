#!/bin/bash
cd "$(dirname "$0")/.."
for v in ${VARIANTS:-0 2 1}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --scan-variant $v > gpurun_out/scanvar_$v.log 2>&1 || exit $?
  grep '^{' gpurun_out/scanvar_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('variant', $v, d['value'], 'q/s', d['roofline']['achieved'], 'GB/s', d['roofline']['avg_launch_ms'], 'ms')"
done
