// Row LayerNorm helpers shared by the encoder kernels and the GEMM's fused split-K + LayerNorm
// finish (one wave per row, H = 64 * EPL, EPL a multiple of 4 and <= 16).
#pragma once
#include "drt_common.h"

namespace drt {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int EPL>
__device__ __forceinline__ void ln_row(float (&x)[EPL], const float* gamma, const float* beta, float eps, int lane,
                                       int H, __bf16* out_row) {
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < EPL; ++e) s += x[e];
  const float mean = wave_sum(s) / (float)H;
  float v = 0.f;
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const float d = x[e] - mean;
    v += d * d;
  }
  const float var = wave_sum(v) / (float)H;
  const float rstd = rsqrtf(var + eps);
  // element e of lane: column c = (e / 4) * 256 + lane * 4 + (e % 4)   (4-wide chunks)
#pragma unroll
  for (int e4 = 0; e4 < EPL / 4; ++e4) {
    const int c = e4 * 256 + lane * 4;
    bf16x4 o;
#pragma unroll
    for (int u = 0; u < 4; ++u) o[u] = (__bf16)((x[e4 * 4 + u] - mean) * rstd * gamma[c + u] + beta[c + u]);
    *(bf16x4*)(out_row + c) = o;
  }
}

// ln_row with gamma / beta already in registers (g[e], b[e] of column (e / 4) * 256 + lane * 4 + e % 4):
// the same arithmetic in the same order, for kernels that normalise many rows per wave.
template <int EPL>
__device__ __forceinline__ void ln_row_gb(float (&x)[EPL], const float (&g)[EPL], const float (&b)[EPL], float eps,
                                          int lane, int H, __bf16* out_row) {
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < EPL; ++e) s += x[e];
  const float mean = wave_sum(s) / (float)H;
  float v = 0.f;
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const float d = x[e] - mean;
    v += d * d;
  }
  const float var = wave_sum(v) / (float)H;
  const float rstd = rsqrtf(var + eps);
#pragma unroll
  for (int e4 = 0; e4 < EPL / 4; ++e4) {
    const int c = e4 * 256 + lane * 4;
    bf16x4 o;
#pragma unroll
    for (int u = 0; u < 4; ++u) o[u] = (__bf16)((x[e4 * 4 + u] - mean) * rstd * g[e4 * 4 + u] + b[e4 * 4 + u]);
    *(bf16x4*)(out_row + c) = o;
  }
}

}  // namespace drt
