#!/bin/bash
# PMC passes over the small post-scan kernels (tools/merge_bench.py).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmcs_1 -o run -- python3 $R/tools/merge_bench.py > $R/gpurun_out/pmcs_1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d $R/gpurun_out/pmcs_2 -o run -- python3 $R/tools/merge_bench.py > $R/gpurun_out/pmcs_2.log 2>&1 || exit $?
