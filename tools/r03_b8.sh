#!/bin/bash
# Round 3 session B8/B9: attention backward A/B (product library vs a variant, checksums), then
# the attention / tower gradient tests on the product library.
#   VARIANT=<name of denseretrievaltoolkits_amd/variants/libdrt_hip.<name>.so>  TAG=<log tag>
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${TAG:-r03i}
timeout -k 10 200 python3 tools/attn_bwd_probe.py > $OUT/attn_${TAG}_new.log 2>&1; rc=$?; echo "new rc=$rc"; tail -1 $OUT/attn_${TAG}_new.log; [ $rc -ne 0 ] && exit $rc
DRT_LIB=$R/denseretrievaltoolkits_amd/variants/libdrt_hip.${VARIANT}.so timeout -k 10 200 python3 tools/attn_bwd_probe.py > $OUT/attn_${TAG}_${VARIANT}.log 2>&1; rc=$?; echo "$VARIANT rc=$rc"; tail -1 $OUT/attn_${TAG}_${VARIANT}.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_encoder_bwd_gpu.py tests/test_train_tower_gpu.py > $OUT/tests_${TAG}.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_${TAG}.log
exit $rc
