// Backward building blocks of the bi-encoder tower (the training step of
// run_random_sampling.py, DRT/trainer/trainer.py:113-133 -> DRModel.forward -> HF BertModel
// under autograd).  Each kernel restates the gradient of one forward op of
// transformers modeling_bert.py (BertSelfOutput / BertOutput LayerNorm :282-352,
// BertIntermediate GELU :325-337, nn.Linear bias) for the bf16 activations the HIP forward
// stores; the tower-level assembly (and attention backward) is the next step.
//
//   layernorm_bwd   dx = rstd (g - mean(g) - xhat mean(g xhat)),  g = dy * gamma,
//                   (+ a residual gradient), per-block dgamma / dbeta partials
//   colsum          out[n] = sum_rows x[row][n] in a fixed order (bias / LN parameter grads)
//   gelu_bwd        dx = dy (Phi(x) + x phi(x))      (erf GELU, activations.py:70-90)
//   transpose_bf16  y[c][r] = x[r][c]                 (operand layout for weight gradients)
#include "drt_common.h"

namespace drt {

__device__ __forceinline__ float bwd_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int kLnBwdBlocks = 1024;   // grid of the row pass = rows of the parameter-gradient partials

// One wave per row (grid-stride over rows), H = 64 * EPL; lane owns columns
// (e / 4) * 256 + lane * 4 + e % 4.  Statistics recomputed from the stored bf16 pre-LN sums
// exactly as layernorm_bf16_kernel computed them.  Each block leaves its dgamma / dbeta
// partial sums in part[blockIdx.x][0..H) and part[gridDim.x + blockIdx.x][0..H).
template <int EPL>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const __bf16* dy, const __bf16* x, const float* gamma,
                                                            float eps, int64_t M, int H, const __bf16* dres,
                                                            __bf16* dx, float* part) {
  __shared__ float red[4][2][EPL * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float dg[EPL], db[EPL], gm[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    dg[e] = 0.f;
    db[e] = 0.f;
    gm[e] = gamma[(e >> 2) * 256 + lane * 4 + (e & 3)];
  }
  for (int64_t t = (int64_t)blockIdx.x * 4 + wave; t < M; t += (int64_t)gridDim.x * 4) {
    float xv[EPL], gv[EPL], dyv[EPL];
#pragma unroll
    for (int e4 = 0; e4 < EPL / 4; ++e4) {
      const int c = e4 * 256 + lane * 4;
      const bf16x4 a = *(const bf16x4*)(x + t * H + c);
      const bf16x4 b = *(const bf16x4*)(dy + t * H + c);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        xv[e4 * 4 + u] = (float)a[u];
        dyv[e4 * 4 + u] = (float)b[u];
      }
    }
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) s += xv[e];
    const float mean = bwd_wave_sum(s) / (float)H;
    float v = 0.f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const float d = xv[e] - mean;
      v += d * d;
    }
    const float rstd = rsqrtf(bwd_wave_sum(v) / (float)H + eps);
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      xv[e] = (xv[e] - mean) * rstd;   // xhat
      gv[e] = dyv[e] * gm[e];
      sg += gv[e];
      sgx += gv[e] * xv[e];
      dg[e] += dyv[e] * xv[e];
      db[e] += dyv[e];
    }
    const float mg = bwd_wave_sum(sg) / (float)H, mgx = bwd_wave_sum(sgx) / (float)H;
#pragma unroll
    for (int e4 = 0; e4 < EPL / 4; ++e4) {
      const int c = e4 * 256 + lane * 4;
      bf16x4 r = {};
      if (dres) r = *(const bf16x4*)(dres + t * H + c);
      bf16x4 o;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e4 * 4 + u;
        o[u] = (__bf16)(rstd * (gv[e] - mg - xv[e] * mgx) + (dres ? (float)r[u] : 0.f));
      }
      *(bf16x4*)(dx + t * H + c) = o;
    }
  }
  // fixed-order block reduction of the 4 waves' parameter-gradient sums
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    red[wave][0][e * 64 + lane] = dg[e];
    red[wave][1][e * 64 + lane] = db[e];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < EPL * 64; i += 256) {
    const int e = i >> 6, ln = i & 63;
    const int col = (e >> 2) * 256 + ln * 4 + (e & 3);
    part[(int64_t)blockIdx.x * H + col] = ((red[0][0][i] + red[1][0][i]) + red[2][0][i]) + red[3][0][i];
    part[(int64_t)(gridDim.x + blockIdx.x) * H + col] = ((red[0][1][i] + red[1][1][i]) + red[2][1][i]) + red[3][1][i];
  }
}

// out[n] = sum over rows [0, M) of x[row][n]: stage 1 (this kernel with FINAL = false) sums
// row slabs into part[slab][n]; stage 2 (FINAL = true) sums the slabs in order.  fp32 sums.
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* x, int64_t M, int64_t N, int64_t rows_per,
                                                     float* out) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = r0 + rows_per < M ? r0 + rows_per : M;
  float s = 0.f;
  for (int64_t r = r0; r < r1; ++r) s += (float)x[r * N + n];
  out[(int64_t)blockIdx.y * N + n] = s;
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const __bf16* dy, const __bf16* pre, int64_t n, __bf16* dx) {
  const int64_t i8 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i8 >= n) return;
  if (i8 + 8 <= n) {
    const bf16x8 g = *(const bf16x8*)(dy + i8);
    const bf16x8 xv = *(const bf16x8*)(pre + i8);
    bf16x8 o;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float x = (float)xv[u];
      const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
      const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
      o[u] = (__bf16)((float)g[u] * (cdf + x * pdf));
    }
    *(bf16x8*)(dx + i8) = o;
  } else {
    for (int64_t i = i8; i < n; ++i) {
      const float x = (float)pre[i];
      const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
      const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
      dx[i] = (__bf16)((float)dy[i] * (cdf + x * pdf));
    }
  }
}

// 64 x 64 tiles through LDS (padded rows: conflict-free column reads).
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const __bf16* x, int64_t R, int64_t C, __bf16* y) {
  __shared__ __bf16 t[64][66];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    t[i][tx] = (r < R && c < C) ? x[r * C + c] : (__bf16)0.0f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < C && r < R) y[c * R + r] = t[tx][i];
  }
}

static int64_t colsum_slabs(int64_t M) { return M < 256 ? 1 : (M + 255) / 256 < 512 ? (M + 255) / 256 : 512; }

template <typename T>
static int colsum_launch(const T* x, int64_t M, int64_t N, float* out, float* ws, hipStream_t s) {
  const int64_t slabs = colsum_slabs(M);
  const int64_t rows_per = (M + slabs - 1) / slabs;
  const unsigned gx = (unsigned)((N + 255) / 256);
  if (slabs == 1) {
    hipLaunchKernelGGL(colsum_kernel<T>, dim3(gx, 1), dim3(256), 0, s, x, M, N, M, out);
  } else {
    hipLaunchKernelGGL(colsum_kernel<T>, dim3(gx, (unsigned)slabs), dim3(256), 0, s, x, M, N, rows_per, ws);
    hipLaunchKernelGGL(colsum_kernel<float>, dim3(gx, 1), dim3(256), 0, s, (const float*)ws, slabs, N, slabs, out);
  }
  return hip_status(hipGetLastError());
}

}  // namespace drt

using namespace drt;

extern "C" {

size_t drt_colsum_workspace(int64_t M, int64_t N) {
  if (M <= 0 || N <= 0) return 0;
  const int64_t slabs = colsum_slabs(M);
  return slabs > 1 ? (size_t)slabs * (size_t)N * sizeof(float) : 0;
}

int drt_colsum_bf16(const void* x, int64_t M, int64_t N, float* out, void* ws, size_t ws_bytes, void* stream) {
  DRT_REQUIRE(M >= 0 && N >= 0);
  if (N == 0) return DRT_OK;
  DRT_REQUIRE(out);
  hipStream_t s = (hipStream_t)stream;
  if (M == 0) return hip_status(hipMemsetAsync(out, 0, N * sizeof(float), s));
  DRT_REQUIRE(x && ws_bytes >= drt_colsum_workspace(M, N) && (ws || drt_colsum_workspace(M, N) == 0));
  return colsum_launch<__bf16>((const __bf16*)x, M, N, out, (float*)ws, s);
}

size_t drt_layernorm_bwd_workspace(int64_t M, int32_t H) {
  if (M <= 0 || H <= 0) return 0;
  return (size_t)2 * kLnBwdBlocks * (size_t)H * sizeof(float) + drt_colsum_workspace(kLnBwdBlocks, 2 * H);
}

// dx = LN backward of dy through out = LN(x) (gamma; x = the bf16 pre-LN sums the forward
// stored) + dres (residual gradient, may be NULL); dgamma / dbeta fp32 [H] (deterministic).
int drt_layernorm_bwd_bf16(const void* dy, const void* x, const float* gamma, float eps, int64_t M, int32_t H,
                           const void* dres, void* dx, float* dgamma, float* dbeta, void* ws, size_t ws_bytes,
                           void* stream) {
  DRT_REQUIRE(M > 0 && H > 0 && H % 256 == 0 && H <= 1024);
  DRT_REQUIRE(dy && x && gamma && dx && dgamma && dbeta && ws && ws_bytes >= drt_layernorm_bwd_workspace(M, H));
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)ws;   // [2 * blocks][H]: dgamma rows then dbeta rows
  const dim3 grid(kLnBwdBlocks);
#define LNB(E) hipLaunchKernelGGL(layernorm_bwd_kernel<E>, grid, dim3(256), 0, s, (const __bf16*)dy, (const __bf16*)x, \
                                  gamma, eps, M, (int)H, (const __bf16*)dres, (__bf16*)dx, part)
  switch (H / 64) {
    case 4: LNB(4); break;
    case 8: LNB(8); break;
    case 12: LNB(12); break;
    case 16: LNB(16); break;
    default: return DRT_EINVAL;
  }
#undef LNB
  float* ws2 = part + (size_t)2 * kLnBwdBlocks * H;
  int rc = colsum_launch<float>(part, kLnBwdBlocks, H, dgamma, ws2, s);
  if (rc) return rc;
  return colsum_launch<float>(part + (size_t)kLnBwdBlocks * H, kLnBwdBlocks, H, dbeta, ws2, s);
}

int drt_gelu_bwd_bf16(const void* dy, const void* pre, int64_t n, void* dx, void* stream) {
  DRT_REQUIRE(n >= 0);
  if (n == 0) return DRT_OK;
  DRT_REQUIRE(dy && pre && dx);
  const int64_t blocks = (n + 2047) / 2048;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const __bf16*)dy,
                     (const __bf16*)pre, n, (__bf16*)dx);
  return hip_status(hipGetLastError());
}

int drt_transpose_bf16(const void* x, int64_t R, int64_t C, void* y, void* stream) {
  DRT_REQUIRE(R >= 0 && C >= 0);
  if (R == 0 || C == 0) return DRT_OK;
  DRT_REQUIRE(x && y);
  dim3 grid((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64));
  hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const __bf16*)x, R, C,
                     (__bf16*)y);
  return hip_status(hipGetLastError());
}

}  // extern "C"
