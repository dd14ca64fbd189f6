#!/bin/bash
# Round 3 session B22: one-launch sample threshold (kth_rank_kernel) -- search / distributed-search
# tests incl. the white-box tau test, then the headline bench (search only) A/B against the previous
# search build (variant shead), alternating; then the GEMM-threshold A/B of tools/r03_b21.sh.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${TAG:-r03zm}
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_search_gpu.py tests/test_dist_search_gpu.py > $OUT/tests_$TAG.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
V=$R/denseretrievaltoolkits_amd/variants
for i in 1 2; do
  unset DRT_LIB
  timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-encode > $OUT/${TAG}_bench_rank_$i.log 2>&1 || exit 1
  DRT_LIB=$V/libdrt_hip.shead.so timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-encode > $OUT/${TAG}_bench_head_$i.log 2>&1 || exit 1
done
for f in $OUT/${TAG}_bench_*.log; do echo "$(basename $f): $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["uncertified_queries_resolved"])')"; done
TAG=r03zl bash tools/r03_b21.sh
