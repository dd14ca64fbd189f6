#!/bin/bash
# Round 3 session B17 (experiment, reverted): attention backward at NB = 5 with dS^T through LDS (dQ
# units read dS back instead of recomputing both score products) -- gradient tests, then the probe
# A/B against the committed kernel (variant head), alternating.  DESIGN.md §5 records the outcome.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${TAG:-r03zf}
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_encoder_bwd_gpu.py > $OUT/tests_$TAG.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
V=$R/denseretrievaltoolkits_amd/variants
for i in 1 2; do
  timeout -k 10 300 python3 tools/attn_bwd_probe.py > $OUT/${TAG}_probe_dsl_$i.log 2>&1 || exit 1
  DRT_LIB=$V/libdrt_hip.head.so timeout -k 10 300 python3 tools/attn_bwd_probe.py > $OUT/${TAG}_probe_head_$i.log 2>&1 || exit 1
done
for f in $OUT/${TAG}_probe_*.log; do echo "$(basename $f): $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v for k, v in d.items() if "L156" in k or "L128" in k})')"; done
