#!/bin/bash
# Global-threshold protocol on one GPU box: parity tests, single-GPU simulation
# of the N-rank step, and a 2-rank gloo rehearsal of bench.py's N > 1 logic.
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python -m pytest ${TEST_PATHS:-tests/test_dist_search_gpu.py} -m gpu -q -rfE --timeout 600 > $OUT/dist_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/dist_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
timeout -k 10 600 python tools/sim_dist.py --world ${WORLD:-8} --steps 20 --check > $OUT/sim_dist.log 2>&1 || { echo "sim rc=$?"; tail -20 $OUT/sim_dist.log; exit 3; }
tail -1 $OUT/sim_dist.log
DRT_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --n-corpus 2000000 \
  > $OUT/gloo2.log 2>&1 || { echo "gloo rc=$?"; tail -20 $OUT/gloo2.log; exit 4; }
grep '^{' $OUT/gloo2.log | cut -c1-300
for st in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --streams $st --n-corpus ${NC:-10000000} > $OUT/bench_s$st.log 2>&1 || exit 5
  grep '^{' $OUT/bench_s$st.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams', $st, d['value'], 'q/s', d['ms_per_step'], 'ms/step scan', d['roofline']['avg_launch_ms'])"
done
