set -u
mkdir -p gpurun_out
V=denseretrievaltoolkits_amd/variants
for r in 1 2 3; do
  for v in ${VARIANTS:-prod stg2 stg4 stg8}; do
    if [ $v = prod ]; then L=denseretrievaltoolkits_amd/libdrt_hip.so; else L=$V/libdrt_hip.$v.so; fi
    out=$(DRT_LIB=$L timeout -k 10 120 python3 tools/scan_group_pmc.py --reps 20 2>/dev/null | grep '^{') || { echo "FAIL $v"; exit 1; }
    echo "$r $v $out" | tee -a gpurun_out/${ABOUT:-stg_ab}.txt
  done
done
