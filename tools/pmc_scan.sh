#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cd /tmp
for v in ${VARIANTS:-0 3}; do
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcscan_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --scan-variant $v > $GRAFT_REPO_ROOT/gpurun_out/pmcscan_$v.log 2>&1 || exit $?
  echo "variant $v rc=$?"
done
