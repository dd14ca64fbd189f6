#!/bin/bash
# training-path GPU check: encoder backward / tower / golden training tests, then the C3 step
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_encoder_bwd_gpu.py tests/test_train_tower_gpu.py tests/test_golden_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_h.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_h.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -c "import sys, json, torch; sys.path.insert(0, '.'); import bench_legs as bench_encode; print(json.dumps(bench_encode.run_train_step(torch.device('cuda', 0), steps=5)))" > gpurun_out/train_h.log 2>&1 || exit $?
tail -1 gpurun_out/train_h.log
