#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench -> rocprof stats.
# Stops at the first crash / abort / timeout (exit status other than 0/1 from
# pytest, non-zero elsewhere); plain test failures (exit 1) still let the
# measurement steps run.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEPS=${STEPS:-20}
TAG=${TAG:-r01}

run() {  # run <name> <timeout> cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session.log
  timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session.log
  tail -n 30 $OUT/$name.log
  return $rc
}

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  run pytest_gpu ${TEST_TIMEOUT:-900} python -u -m pytest ${TEST_PATHS:-tests} -m gpu -v -rfE --timeout 600 --timeout-method thread ${PYTEST_ARGS:-}
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: pytest rc=$rc"; exit $rc; fi
fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench ${BENCH_TIMEOUT:-900} python -u bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS:-} || exit $?
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench_$TAG.json
if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp
  run_prof() {
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_$TAG -o run --output-format csv \
      -- python3 $GRAFT_REPO_ROOT/bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-evaluate > $GRAFT_REPO_ROOT/$OUT/prof_$TAG.log 2>&1
  }
  run_prof; rc=$?
  echo "=== rocprof rc=$rc" | tee -a $GRAFT_REPO_ROOT/$OUT/session.log
  find $GRAFT_REPO_ROOT/$OUT/prof_$TAG -name "*stats*" | head
fi
if [ "${PMC:-0}" = "1" ]; then
  cd /tmp
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/$OUT/pmc_${TAG}_$C -o run \
      -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/$OUT/pmc_${TAG}_$C.log 2>&1
    rc=$?; echo "=== pmc $C rc=$rc" | tee -a $GRAFT_REPO_ROOT/$OUT/session.log
    [ $rc -ne 0 ] && exit $rc
  done
  python3 $GRAFT_REPO_ROOT/tools/pmc_traffic.py $GRAFT_REPO_ROOT/$OUT/pmc_${TAG}_FETCH_SIZE $GRAFT_REPO_ROOT/$OUT/pmc_${TAG}_WRITE_SIZE \
    $GRAFT_REPO_ROOT/$OUT/${TAG}_pmc_traffic.json --n-corpus ${NCORPUS:-10000000}
  cd $GRAFT_REPO_ROOT
fi
if [ "${GEMMB:-0}" = "1" ]; then
  cd $GRAFT_REPO_ROOT && timeout -k 10 300 python tools/gemm_bench.py > $OUT/gemm_bench.log 2>&1; echo "=== gemm_bench rc=$?"; tail -2 $OUT/gemm_bench.log
fi
