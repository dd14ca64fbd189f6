#!/bin/bash
# Round 3 session B2: kernel-trace stats of the bench (search + encode legs), per-kernel stats of
# the two training steps (C3 shape and the run.sh recipe shape), and PMC passes over attention.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_r03b -o run --output-format csv \
  -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-evaluate > $OUT/prof_r03b.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/prof_r03b.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_train_r03b -o run --output-format csv \
  -- python3 $R/tools/train_len.py > $OUT/prof_train_r03b.log 2>&1
rc=$?; echo "rocprof train rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/prof_train_r03b.log; exit $rc; }
timeout -k 10 120 python3 $R/tools/attn_bwd_probe.py > $OUT/attn_probe_r03b.log 2>&1
rc=$?; echo "attn probe rc=$rc"; tail -2 $OUT/attn_probe_r03b.log; [ $rc -ne 0 ] && exit $rc
bash $R/tools/pmc_attn.sh
