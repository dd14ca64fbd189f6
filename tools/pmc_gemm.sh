#!/bin/bash
# PMC passes over one GEMM variant (separate rocprofv3 run per counter group).
# env: VARIANTS (default 7), SHAPE "N K FLAGS" (default "2304 768 0"), PMC_GROUPS (";"-separated counter lists)
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_gemm
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
PMC_GROUPS_DEF="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE;SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS"
IFS=';' read -ra GR <<< "${PMC_GROUPS:-$PMC_GROUPS_DEF}"
i=0
for C in "${GR[@]}"; do
  for V in ${VARIANTS:-7}; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/p${i}_v$V -o run -- python3 $R/tools/gemm_one.py $V ${SHAPE:-2304 768 0} > $OUT/p${i}_v$V.log 2>&1
    rc=$?; echo "pass $i v$V rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
  i=$((i+1))
done
python3 - <<'PY'
import csv, glob, os, collections
R=os.environ["GRAFT_REPO_ROOT"]
for f in sorted(glob.glob(R+"/gpurun_out/pmc_gemm/*/run_counter_collection.csv")):
    acc=collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        if "gemm" not in row.get("Kernel_Name",""): continue
        acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    print(f.split("/")[-2], {k: round(sum(v)/len(v)) for k,v in acc.items()})
PY
