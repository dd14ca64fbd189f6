#!/bin/bash
# Round 3 session B6: query tower split-K targets (product 512 blocks vs 64 vs no split) and the
# attention probe of the product build (5-wave dropout forward at 4 WGs/CU).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
for v in split64 nosplit; do
  DRT_LIB=$R/denseretrievaltoolkits_amd/variants/libdrt_hip.$v.so timeout -k 10 200 python3 tools/query_encode.py > $OUT/qenc_r03f_$v.log 2>&1
  rc=$?; echo "qenc $v rc=$rc"; tail -1 $OUT/qenc_r03f_$v.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 python3 tools/query_encode.py > $OUT/qenc_r03f.log 2>&1
rc=$?; echo "qenc product rc=$rc"; tail -1 $OUT/qenc_r03f.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 tools/attn_bwd_probe.py > $OUT/attn_probe_r03f.log 2>&1
rc=$?; echo "attn rc=$rc"; tail -1 $OUT/attn_probe_r03f.log; exit $rc
