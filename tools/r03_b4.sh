#!/bin/bash
# Round 3 session B4: pairwise attention-dropout hash (forward) + one-round staging in the attention
# backward (lse / mask / keep words with the row loads; hash-drawn words in staging instead of the
# retired hash kernel): correctness, then timing of attention and the two training steps.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest -m gpu -v -rfE --timeout 300 --timeout-method thread \
  tests/test_encoder_bwd_gpu.py tests/test_train_tower_gpu.py \
  "tests/test_multirank_gpu.py::test_ddp_train_step_world2_matches_single_process" > $OUT/b4_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 $OUT/b4_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 tools/attn_bwd_probe.py > $OUT/attn_probe_r03d.log 2>&1
rc=$?; echo "attn probe rc=$rc"; tail -1 $OUT/attn_probe_r03d.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/train_len.py > $OUT/train_len_r03d.log 2>&1
rc=$?; echo "train rc=$rc"; grep hip_ms $OUT/train_len_r03d.log | cut -c1-400; exit $rc
