#!/bin/bash
# dist-protocol GPU tests + the N = 8 per-rank step simulation (+ its rocprof kernel trace)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist_search_gpu.py tests/test_torch_ops_gpu.py tests/test_multirank_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo "dist tests rc=$rc"; tail -3 gpurun_out/pytest_dist.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/sim_dist.py --world 8 --steps 30 --graph --check > gpurun_out/sim8.log 2>&1 || exit $?
tail -1 gpurun_out/sim8.log
WORLD=8 bash tools/sim_prof.sh > gpurun_out/sim_prof.txt 2>&1; echo "sim_prof rc=$?"
