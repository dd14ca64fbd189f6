#!/bin/bash
# Round 3 session B10: attention backward ablations (staging without global reads / without the
# two matrix phases) beside the product kernel.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for v in product noload nophase; do
  if [ $v = product ]; then L=$R/denseretrievaltoolkits_amd/libdrt_hip.so; else L=$R/denseretrievaltoolkits_amd/variants/libdrt_hip.$v.so; fi
  DRT_LIB=$L timeout -k 10 200 python3 tools/attn_bwd_probe.py > $OUT/attn_r03l_$v.log 2>&1; rc=$?; echo "$v rc=$rc"; tail -1 $OUT/attn_r03l_$v.log | cut -c1-900; [ $rc -ne 0 ] && exit $rc
done
exit 0
