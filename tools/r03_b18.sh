#!/bin/bash
# Round 3 session B18: split-K GEMMs finished in the same launch (last split to arrive per tile,
# gemm_nt_kernel PART + arrival words) -- the split / linear-LN / encoder tests, then the query
# tower A/B against the previous two-launch build (variant head), alternating.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${TAG:-r03zh}
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_encoder_gpu.py > $OUT/tests_$TAG.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
V=$R/denseretrievaltoolkits_amd/variants
for i in 1 2; do
  timeout -k 10 300 python3 tools/query_encode.py > $OUT/${TAG}_qenc_fin_$i.log 2>&1 || exit 1
  DRT_LIB=$V/libdrt_hip.head.so timeout -k 10 300 python3 tools/query_encode.py > $OUT/${TAG}_qenc_head_$i.log 2>&1 || exit 1
done
for f in $OUT/${TAG}_qenc_*.log; do echo "$(basename $f): $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({b: d[b]["eager_ms_per_batch"] for b in ("b8","b128","b512")}, {b: d[b]["graph_ms_per_batch"] for b in ("b8","b128")})')"; done
