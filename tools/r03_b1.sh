#!/bin/bash
# Round 3 session B1: the changed GPU tests, then the full default bench (C2 leg, CPU baselines).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -v -rfE --timeout 300 --timeout-method thread \
  tests/test_multirank_gpu.py tests/test_encoder_bwd_gpu.py tests/test_train_tower_gpu.py tests/test_encoder_gpu.py \
  tests/test_golden_gpu.py > $OUT/b1_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/b1_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py > $OUT/b1_bench.log 2>&1
rc=$?
echo "bench rc=$rc"; grep '^{' $OUT/b1_bench.log | tail -1 > $OUT/bench_r03b.json; tail -c 3000 $OUT/b1_bench.log
exit $rc
