#!/bin/bash
# Round 3 session B14: 128^2 GEMM epilogue through LDS -- query tower A/B (product vs the previous
# gemm.hip as a variant library, interleaved twice), then the GEMM / encoder GPU tests.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${TAG:-r03v}
for rep in 1 2; do
  for v in product prevgemm; do
    if [ $v = product ]; then L=$R/denseretrievaltoolkits_amd/libdrt_hip.so; else L=$R/denseretrievaltoolkits_amd/variants/libdrt_hip.$v.so; fi
    DRT_LIB=$L timeout -k 10 200 python3 tools/query_encode.py > $OUT/qenc_${TAG}_${v}_$rep.log 2>&1; rc=$?; echo "$v $rep rc=$rc"; tail -1 $OUT/qenc_${TAG}_${v}_$rep.log | cut -c1-420; [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_encoder_gpu.py tests/test_encoder_bwd_gpu.py tests/test_train_tower_gpu.py tests/test_golden_gpu.py > $OUT/tests_$TAG.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log
exit $rc
