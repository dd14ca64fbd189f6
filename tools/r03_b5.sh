#!/bin/bash
# Round 3 session B5: 128^2 GEMM with a 4-stage ring for one-round grids + full-tile epilogue
# without per-element guarded loads -- correctness, query tower (product, split-target-256 variant),
# rocprof of the query tower, attention probe of the forward-dropout occupancy variant.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest -m gpu -v -rfE --timeout 300 --timeout-method thread \
  tests/test_encoder_gpu.py tests/test_golden_gpu.py tests/test_trainer_gpu.py > $OUT/b5_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 $OUT/b5_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 tools/query_encode.py > $OUT/qenc_r03e.log 2>&1
rc=$?; echo "qenc rc=$rc"; tail -1 $OUT/qenc_r03e.log | cut -c1-700; [ $rc -ne 0 ] && exit $rc
DRT_LIB=$R/denseretrievaltoolkits_amd/variants/libdrt_hip.split256.so timeout -k 10 200 python3 tools/query_encode.py > $OUT/qenc_r03e_split256.log 2>&1
rc=$?; echo "qenc split256 rc=$rc"; tail -1 $OUT/qenc_r03e_split256.log | cut -c1-700; [ $rc -ne 0 ] && exit $rc
DRT_LIB=$R/denseretrievaltoolkits_amd/variants/libdrt_hip.minb4.so timeout -k 10 120 python3 tools/attn_bwd_probe.py > $OUT/attn_probe_r03e_minb4.log 2>&1
rc=$?; echo "attn minb4 rc=$rc"; tail -1 $OUT/attn_probe_r03e_minb4.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 bash tools/qenc_prof.sh
