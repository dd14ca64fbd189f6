#!/bin/bash
# search-path GPU check: search / multi-rank / dist / op tests, the N = 8 per-rank simulation
# (grouped vs per-batch protocol), and bench.py N = 1 grouped vs per-batch (same box).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py tests/test_multirank_gpu.py tests/test_dist_search_gpu.py tests/test_torch_ops_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_f.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_f.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/sim_dist.py --world 8 --steps 32 --check > gpurun_out/sim8f.log 2>&1 || exit $?
tail -1 gpurun_out/sim8f.log
timeout -k 10 400 python bench.py --steps 32 --warmup 3 --no-encode --no-cpu-baseline --group-queries 2048 > gpurun_out/bench_f.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_f.log | tail -1
timeout -k 10 400 python bench.py --steps 32 --warmup 3 --no-encode --no-cpu-baseline --group-queries 0 > gpurun_out/bench_f0.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_f0.log | tail -1
