#!/bin/bash
# Round 3 session B16: answer matching on the GPU -- tests (device matcher vs host, Trainer.evaluate
# W = 1 / 2), then the C2 evaluate leg.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${TAG:-r03zb}
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_answers_gpu.py tests/test_trainer_gpu.py tests/test_multirank_gpu.py > $OUT/tests_$TAG.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -c "import sys, json, torch; sys.path.insert(0, '$R'); import bench_legs as b; print(json.dumps(b.run_evaluate_c2(torch.device('cuda', 0))))" > $OUT/c2_$TAG.log 2>&1; rc=$?; echo "c2 rc=$rc"; tail -1 $OUT/c2_$TAG.log | cut -c1-1200
exit $rc
