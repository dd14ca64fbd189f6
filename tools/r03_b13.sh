#!/bin/bash
# Round 3 session B13: attention forward rewrite -- probe, then the encoder / training / golden GPU tests.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${TAG:-r03r}
timeout -k 10 200 python3 tools/attn_bwd_probe.py > $OUT/attn_$TAG.log 2>&1; rc=$?; echo "probe rc=$rc"; tail -1 $OUT/attn_$TAG.log | cut -c1-1500; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_encoder_gpu.py tests/test_encoder_bwd_gpu.py tests/test_train_tower_gpu.py tests/test_golden_gpu.py > $OUT/tests_$TAG.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log
exit $rc
