set -u
mkdir -p gpurun_out
V=denseretrievaltoolkits_amd/variants/libdrt_hip.pr5p.so
P=denseretrievaltoolkits_amd/libdrt_hip.so
# correctness first, short limits: one tile per work-group (M 4096), then the persistent loop (M 32768)
DRT_LIB=$V timeout -k 10 60 python3 tools/gemm_abl_time.py 4096 3 2>&1 | grep '^{' | tee -a gpurun_out/pr5p_ab.txt || exit 1
DRT_LIB=$P timeout -k 10 60 python3 tools/gemm_abl_time.py 4096 3 2>&1 | grep '^{' | tee -a gpurun_out/pr5p_ab.txt || exit 1
DRT_LIB=$V timeout -k 10 60 python3 tools/gemm_abl_time.py 32768 3 2>&1 | grep '^{' | tee -a gpurun_out/pr5p_ab.txt || exit 1
for r in 1 2 3; do
  for L in $P $V; do
    DRT_LIB=$L timeout -k 10 120 python3 tools/gemm_abl_time.py 32768 20 2>&1 | grep '^{' | tee -a gpurun_out/pr5p_ab.txt || exit 1
  done
done
for r in 1 2; do
  for L in $P $V; do
    DRT_LIB=$L timeout -k 10 200 python3 tools/ln_ab.py 2>/dev/null | grep '^{' | tee -a gpurun_out/pr5p_enc.txt || exit 1
  done
done
