// Diagnostic (tools/mfma_numerics.py): what one v_mfma_f32_16x16x32_bf16 and a chain of them
// compute, bit for bit -- the summation semantics the canonical-order error bound rests on
// (csrc/search.hip, refine_eps).  One wave per trial: acc = C; for s < S: acc = mfma(A_s, B_s, acc).
// Layout (host side restates it): A [T][S][16 m][32 k], B [T][S][16 n][32 k] (bf16 bits),
// C / D [T][16 m][16 n] fp32.  Lane l holds A[m = l % 16][k = 8 (l / 16) + e], B[n = l % 16][same k],
// D[m = 4 (l / 16) + i][n = l % 16].
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void mfma_chain_kernel(const uint16_t* A, const uint16_t* B, const float* C,
                                                        float* D, int S) {
  const int t = blockIdx.x, l = threadIdx.x;
  const int r = l & 15, kg = l >> 4;
  f32x4 acc;
  for (int i = 0; i < 4; ++i) acc[i] = C[(int64_t)t * 256 + (4 * kg + i) * 16 + r];
  for (int s = 0; s < S; ++s) {
    const uint16_t* a = A + (((int64_t)t * S + s) * 16 + r) * 32 + 8 * kg;
    const uint16_t* b = B + (((int64_t)t * S + s) * 16 + r) * 32 + 8 * kg;
    bf16x8 af, bfr;
    for (int e = 0; e < 8; ++e) {
      af[e] = __builtin_bit_cast(__bf16, a[e]);
      bfr[e] = __builtin_bit_cast(__bf16, b[e]);
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i) D[(int64_t)t * 256 + (4 * kg + i) * 16 + r] = acc[i];
}

extern "C" int mfma_chain(const void* A, const void* B, const void* C, void* D, int T, int S, void* stream) {
  hipLaunchKernelGGL(mfma_chain_kernel, dim3(T), dim3(64), 0, (hipStream_t)stream, (const uint16_t*)A,
                     (const uint16_t*)B, (const float*)C, (float*)D, S);
  return (int)hipGetLastError();
}

// v_mfma_f32_32x32x16_bf16 chains: A [T][S][32 m][16 k], B [T][S][32 n][16 k], C / D [T][32 m][32 n].
// Lane l = (r = l & 31, h = l >> 5) holds A[m = r][k = 8 h + e], B[n = r][same k];
// D[m = (i & 3) + 8 (i >> 2) + 4 h][n = r] in register i.
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(64) void mfma32_chain_kernel(const uint16_t* A, const uint16_t* B, const float* C,
                                                          float* D, int S) {
  const int t = blockIdx.x, l = threadIdx.x;
  const int r = l & 31, h = l >> 5;
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = C[(int64_t)t * 1024 + ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r];
  for (int s = 0; s < S; ++s) {
    const uint16_t* a = A + (((int64_t)t * S + s) * 32 + r) * 16 + 8 * h;
    const uint16_t* b = B + (((int64_t)t * S + s) * 32 + r) * 16 + 8 * h;
    bf16x8 af, bfr;
    for (int e = 0; e < 8; ++e) {
      af[e] = __builtin_bit_cast(__bf16, a[e]);
      bfr[e] = __builtin_bit_cast(__bf16, b[e]);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc, 0, 0, 0);
  }
  for (int i = 0; i < 16; ++i) D[(int64_t)t * 1024 + ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[i];
}

extern "C" int mfma32_chain(const void* A, const void* B, const void* C, void* D, int T, int S, void* stream) {
  hipLaunchKernelGGL(mfma32_chain_kernel, dim3(T), dim3(64), 0, (hipStream_t)stream, (const uint16_t*)A,
                     (const uint16_t*)B, (const float*)C, (float*)D, S);
  return (int)hipGetLastError();
}
