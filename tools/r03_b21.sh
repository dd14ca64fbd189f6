#!/bin/bash
# Round 3 session B21: threshold of the 256^2 whole-line GEMM plan (DRT_LARGE_MIN_TILES 128 = product,
# 160 / 200 = variants) on the query tower (batch 8 / 128 / 512 x 32 tokens) and the encode leg, alternating.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${TAG:-r03zl}
V=$R/denseretrievaltoolkits_amd/variants
for i in 1 2; do
  for v in product lmt160 lmt200; do
    if [ $v = product ]; then unset DRT_LIB; else export DRT_LIB=$V/libdrt_hip.$v.so; fi
    timeout -k 10 300 python3 tools/query_encode.py > $OUT/${TAG}_qenc_${v}_$i.log 2>&1 || exit 1
  done
done
for f in $OUT/${TAG}_qenc_*.log; do echo "$(basename $f): $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({b: d[b]["eager_ms_per_batch"] for b in ("b8","b128","b512")})')"; done
