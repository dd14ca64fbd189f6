#!/bin/bash
# Round 3 session B12: the relaxed HIP-tower loss test, recipe-step kernel profile, query tower
# per-batch profile.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_golden_gpu.py > $OUT/tests_r03q.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests_r03q.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
GRAFT_REPO_ROOT=$R LEG_ARGS='bq=128, n=8, p_len=156' TAG=_recipe bash tools/train_prof.sh > $OUT/prof_recipe_summary.txt 2>&1; rc=$?; echo "recipe prof rc=$rc"; cat $OUT/prof_recipe_summary.txt | head -40; [ $rc -ne 0 ] && exit $rc
GRAFT_REPO_ROOT=$R bash tools/qenc_prof2.sh > $OUT/prof_qenc2_summary.txt 2>&1; rc=$?; echo "qenc prof rc=$rc"; cat $OUT/prof_qenc2_summary.txt | head -40
exit $rc
