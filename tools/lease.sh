#!/bin/bash
# One parameterised GPU-box session (replaces the per-session scripts of earlier rounds).
#   TAG=r04a bash tools/lease.sh tests smoke bench bench_gloo2 prof_c2 ...
# Steps run in the order given, each under its own time limit; the session stops at the first
# step that fails (no retries).  Logs land in gpurun_out/${TAG}_<step>.log.
# Steps:
#   tests        pytest -m gpu over ${TEST_PATHS:-tests}
#   smoke        __graft_entry__.smoke()
#   bench        the driver's bench line (N = 1), ${BENCH_ARGS}
#   bench_search bench.py search leg only (no encode / evaluate / CPU baseline)
#   bench_gloo2  `bench.py --gpus 2` with no launcher: two ranks on the one GPU over gloo
#   prof_bench   rocprofv3 --kernel-trace --stats of the search-only bench
#   prof_c2      rocprofv3 kernel trace of search_batches over 1M rows (C2 shard size) + trace tail
#   prof_sim8    rocprofv3 kernel trace of the simulated W = 8 per-rank step + trace tail
#   pmc_scan     HBM traffic of the filter scan (FETCH_SIZE / WRITE_SIZE passes); PMC_BENCH_ARGS (bench.py
#                steps / path), PMC_SHAPE_ARGS (pmc_traffic.py --launch-queries Q --launch-rows R: a grouped launch)
#   cmd          run "$CMD" (a python tool invocation) under a 600 s limit
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${TAG:-r04}
cd $R

step() {  # step <name> <timeout> cmd...
  local name=$1 to=$2; shift 2
  echo "=== $TAG $name: $*" | tee -a $OUT/session.log
  timeout -k 10 "$to" "$@" > $OUT/${TAG}_$name.log 2>&1
  local rc=$?
  echo "=== $TAG $name rc=$rc" | tee -a $OUT/session.log
  tail -n ${TAIL:-6} $OUT/${TAG}_$name.log | cut -c1-600
  return $rc
}

prof() {  # prof <name> <timeout> python-args...
  local name=$1 to=$2; shift 2
  ( cd /tmp && timeout -k 10 "$to" rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_$name -o run --output-format csv \
      -- python3 "$@" > $OUT/${TAG}_$name.log 2>&1 )
  local rc=$?
  echo "=== $TAG $name rc=$rc" | tee -a $OUT/session.log
  tail -n 3 $OUT/${TAG}_$name.log | cut -c1-600
  [ $rc -ne 0 ] && return $rc
  python3 $R/tools/trace_tail.py $OUT/${TAG}_$name --last ${LAST:-600} --show ${SHOW:-30} \
    --json $OUT/${TAG}_${name}_tail.json > $OUT/${TAG}_${name}_tail.txt 2>&1
  head -n 14 $OUT/${TAG}_${name}_tail.txt
}

for s in "$@"; do
  case $s in
    tests) step tests ${TEST_TIMEOUT:-900} python3 -u -m pytest ${TEST_PATHS:-tests} -m gpu -v -rfE \
             --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} || exit $? ;;
    smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) step bench ${BENCH_TIMEOUT:-900} python3 -u bench.py --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:-} || exit $?
           grep '^{' $OUT/${TAG}_bench.log | tail -1 > $OUT/${TAG}_bench.json ;;
    bench_search) step bench_search 300 python3 -u bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline \
             --no-encode ${BENCH_ARGS:-} || exit $? ;;
    bench_gloo2) DRT_BENCH_BACKEND=gloo step bench_gloo2 600 python3 -u bench.py --gpus 2 --n-corpus 2000000 \
             --steps 8 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} || exit $? ;;
    prof_bench) prof prof_bench 600 $R/bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-evaluate --no-encode \
                  ${BENCH_ARGS:-} || exit $? ;;
    prof_c2) LAST=${LAST:-800} prof prof_c2 600 $R/tools/search_ab.py --n 1000000 --steps 78 --rounds 2 \
             --groups ${GROUPS_AB:-0,2048} || exit $? ;;
    prof_sim8) prof prof_sim8 600 $R/tools/sim_dist.py --world 8 --steps 20 || exit $? ;;
    pmc_scan) for C in FETCH_SIZE WRITE_SIZE; do
                ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $OUT/${TAG}_pmc_$C -o run \
                    -- python3 $R/bench.py ${PMC_BENCH_ARGS:---steps 3 --warmup 1} --no-cpu-baseline --no-encode \
                    > $OUT/${TAG}_pmc_$C.log 2>&1 )
                rc=$?; echo "=== $TAG pmc $C rc=$rc" | tee -a $OUT/session.log; [ $rc -ne 0 ] && exit $rc
              done
              python3 $R/tools/pmc_traffic.py $OUT/${TAG}_pmc_FETCH_SIZE $OUT/${TAG}_pmc_WRITE_SIZE \
                $OUT/${TAG}_pmc_traffic.json --n-corpus ${NCORPUS:-10000000} ${PMC_SHAPE_ARGS:-} || exit $? ;;
    cmd) step cmd 600 ${CMD} || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
