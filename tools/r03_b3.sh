#!/bin/bash
# Round 3 session B3: register-resident attention backward -- correctness first, then timing,
# then kernel-trace stats of the bench and of the training steps, then PMC passes over attention.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest -m gpu -v -rfE --timeout 300 --timeout-method thread \
  tests/test_encoder_bwd_gpu.py tests/test_train_tower_gpu.py tests/test_golden_gpu.py \
  "tests/test_multirank_gpu.py::test_ddp_train_step_world2_matches_single_process" \
  "tests/test_multirank_gpu.py::test_rrtrainer_evaluate_world2" tests/test_trainer_gpu.py tests/test_encoder_gpu.py \
  "tests/test_search_gpu.py::test_filter_scan_flavours_bit_exact" > $OUT/b3_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 $OUT/b3_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 tools/attn_bwd_probe.py > $OUT/attn_probe_r03c.log 2>&1
rc=$?; echo "attn probe rc=$rc"; tail -1 $OUT/attn_probe_r03c.log; [ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_train_r03c -o run --output-format csv \
  -- python3 $R/tools/train_len.py > $OUT/prof_train_r03c.log 2>&1
rc=$?; echo "rocprof train rc=$rc"; tail -2 $OUT/prof_train_r03c.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_r03c -o run --output-format csv \
  -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-evaluate > $OUT/prof_r03c.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"; grep '^{' $OUT/prof_r03c.log | tail -1 | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash $R/tools/pmc_attn.sh
