#!/bin/bash
# PMC pass over the encode leg (bf16 BERT-base, 512 x 128 tokens): MFMA busy cycles and
# GRBM_GUI_ACTIVE per kernel -> MFMA utilisation and the clock the chip holds under each
# kernel (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE is summed over the 8 XCDs).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_enc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv \
  -d $OUT -o run -- python3 -c "import sys, json, torch; sys.path.insert(0, '$R'); import bench_legs as bench_encode; print(json.dumps(bench_encode.run(torch.device('cuda', 0), steps=2, warmup=1)))" \
  > $OUT/run.log 2>&1
rc=$?
echo "pmc rc=$rc"
[ $rc -ne 0 ] && { tail -5 $OUT/run.log; exit $rc; }
python3 $R/tools/pmc_encode_report.py $OUT > $R/gpurun_out/pmc_enc.json
cat $R/gpurun_out/pmc_enc.json
