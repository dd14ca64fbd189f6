# usage: bash tools/attn_ab.sh <variant> ...   (prod = the in-tree library)
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    if [ $v = prod ]; then L=denseretrievaltoolkits_amd/libdrt_hip.so; else L=denseretrievaltoolkits_amd/variants/libdrt_hip.$v.so; fi
    DRT_LIB=$L timeout -k 10 200 python3 tools/attn_ab.py 2>>gpurun_out/attn_ab.err | grep '^{' | tee -a gpurun_out/attn_ab.txt
  done
done
