#!/bin/bash
# Round 3 session B7: query tower split-K target sweep (32 / 96 / 128 blocks)
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for v in split32 split96 split128; do
  DRT_LIB=$R/denseretrievaltoolkits_amd/variants/libdrt_hip.$v.so timeout -k 10 200 python3 tools/query_encode.py > $OUT/qenc_r03g_$v.log 2>&1
  rc=$?; echo "qenc $v rc=$rc"; tail -1 $OUT/qenc_r03g_$v.log | cut -c1-330; [ $rc -ne 0 ] && exit $rc
done
exit 0
