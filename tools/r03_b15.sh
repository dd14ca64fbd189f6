#!/bin/bash
# Round 3 session B15: bias gradients from the LayerNorm / attention backwards -- GPU tests, then
# the C3 and recipe training legs (ms per step) and a kernel profile of the recipe step.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${TAG:-r03w}
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_encoder_bwd_gpu.py tests/test_train_tower_gpu.py tests/test_golden_gpu.py tests/test_multirank_gpu.py > $OUT/tests_$TAG.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -c "import sys, json, torch; sys.path.insert(0, '$R'); import bench_legs as b; d = torch.device('cuda', 0); print(json.dumps({'c3': b.run_train_step(d), 'recipe': b.run_train_step(d, bq=128, n=8, p_len=156)}))" > $OUT/train_$TAG.log 2>&1; rc=$?; echo "train rc=$rc"; tail -1 $OUT/train_$TAG.log | cut -c1-1500; [ $rc -ne 0 ] && exit $rc
GRAFT_REPO_ROOT=$R LEG_ARGS='bq=128, n=8, p_len=156' TAG=_recipe_$TAG bash tools/train_prof.sh > $OUT/prof_recipe_${TAG}_summary.txt 2>&1; rc=$?; echo "prof rc=$rc"; grep -E "drt::|total" $OUT/prof_recipe_${TAG}_summary.txt | head -24
exit $rc
