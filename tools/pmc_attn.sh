#!/bin/bash
# PMC passes over the attention forward / backward at the C3 and recipe shapes
# (tools/attn_bwd_probe.py): where the backward's cycles go (waves waiting, VALU vs MFMA issue,
# LDS traffic and bank conflicts).  Each pass is its own run (counter-block limits).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_attn
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
pass() {  # pass <name> <counters...>
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$name -o run \
    -- python3 $R/tools/attn_bwd_probe.py 2 > $OUT/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/$name.log; exit $rc; }
  return 0
}
pass p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
pass p2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
python3 $R/tools/pmc_report.py $OUT/p1 $OUT/p2 > $R/gpurun_out/pmc_attn.json
cat $R/gpurun_out/pmc_attn.json
