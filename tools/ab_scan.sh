#!/bin/bash
# A/B of the filter scan: product library vs a variant (DRT_LIB), alternating, one box.
#   TAG=... VARIANT=prevscan bash tools/ab_scan.sh
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
V=$R/denseretrievaltoolkits_amd/variants/libdrt_hip.${VARIANT:-prevscan}.so
TAG=${TAG:-r04ab}
cd $R
for i in 1 2; do
  for lib in new var; do
    if [ $lib = var ]; then export DRT_LIB=$V; else unset DRT_LIB; fi
    timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-encode --no-cpu-baseline ${BENCH_ARGS:-} \
      > $OUT/${TAG}_bench_${lib}_$i.log 2>&1 || exit 1
    timeout -k 10 200 python3 tools/search_ab.py --n 1000000 --steps 78 --rounds 2 ${AB_ARGS:-} \
      > $OUT/${TAG}_c2_${lib}_$i.log 2>&1 || exit 1
  done
done
unset DRT_LIB
for f in $OUT/${TAG}_bench_*.log; do
  echo "$(basename $f): $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
for f in $OUT/${TAG}_c2_*.log; do echo "$(basename $f): $(tail -1 $f)"; done
