// In-batch-negative score matrix + cross entropy (training step).
//
// Reference: DRModel.forward (DRT/model/biencoder.py:107-119)
//   scores = q_reps @ p_reps^T ; target = arange(Bq) * train_n_passages
//   loss   = CrossEntropyLoss(mean)(scores, target) [* world_size if x-device]
// and SimpleContrastiveLoss (DRT/trainer/losses.py:11-17), target stride
// y.size(0) // x.size(0).  The reference is fp32 end to end, so these
// kernels stay fp32: the GEMMs run on the exact-f32 MFMA
// (v_mfma_f32_32x32x2_f32 = a k-ordered fmaf chain), the CE row pass in fp32.
//
//   drt_gemm_nt_f32      C = A . B^T                 (fp32 in / out)
//   drt_ce_fwd           lse_i, mean loss
//   drt_ce_bwd           dS = (softmax(S) - onehot) * g * scale / m
//   drt_transpose_f32    helper for the backward GEMMs (dQ = dS P, dP = dS^T Q)
#include "drt_common.h"

namespace drt {

constexpr int kF32Threads = 256;
constexpr int kFT = 64;    // output tile 64 x 64, one 32 x 32 MFMA tile per wave
constexpr int kFBK = 32;   // k per LDS stage
constexpr int kFPad = kFBK + 1;

__global__ __launch_bounds__(kF32Threads) void gemm_nt_f32_kernel(const float* A, const float* B, float* C,
                                                                  int64_t m, int64_t n, int64_t k, int64_t lda,
                                                                  int64_t ldb, int64_t ldc, float alpha) {
  __shared__ float As[kFT][kFPad];
  __shared__ float Bs[kFT][kFPad];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.y * kFT, n0 = (int64_t)blockIdx.x * kFT;
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.0f;

  for (int64_t k0 = 0; k0 < k; k0 += kFBK) {
    // stage 64 x 32 of A and of B (8 elements per thread each)
    for (int i = tid; i < kFT * kFBK; i += kF32Threads) {
      const int row = i / kFBK, col = i % kFBK;
      const int64_t gk = k0 + col;
      const int64_t ga = m0 + row, gb = n0 + row;
      As[row][col] = (ga < m && gk < k) ? A[ga * lda + gk] : 0.0f;
      Bs[row][col] = (gb < n && gk < k) ? B[gb * ldb + gk] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < kFBK / 2; ++s) {
      const float a = As[wm * 32 + r][2 * s + h];
      const float b = Bs[wn * 32 + r][2 * s + h];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int64_t row = m0 + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
    const int64_t col = n0 + wn * 32 + r;
    if (row < m && col < n) C[row * ldc + col] = acc[e] * alpha;
  }
}


// ---------------------------------------------------------------------------
// General-layout exact-f32 GEMM for the score matrix and its backward:
//   C[m][n] (+)= sum_k A(m, k) B(k, n)
// A_KC: A stored [m][k] (k contiguous, q / dS) else [k][m] (dS^T operand of dP);
// B_KC: B stored [n][k] (p in the forward) else [k][n] (p / q in the backward).
// 64 x 64 tile per 256-thread block (4 waves x one 32 x 32 v_mfma_f32_32x32x2_f32
// tile), BK = 32, both operands staged k-major in LDS ([k][64 + 4]) so every MFMA
// operand read is one conflict-free ds_read_b32; next k-tile loaded into
// registers (float4 when aligned) while the current one is multiplied.
// Split-K (blockIdx.z) writes partial sums to a workspace that
// splitk_reduce_kernel adds in a fixed order (deterministic, no atomics).
// ---------------------------------------------------------------------------
constexpr int kGT = 64, kGBK = 32, kGLd = kGT + 4;

template <bool KC, bool VEC>
__device__ __forceinline__ void load_op(const float* X, int64_t ld, int64_t r0, int64_t rows, int64_t k0, int64_t kend,
                                        int tid, float (&v)[8]) {
  // KC: tile = 64 rows x 32 k from X[row][k]; else 32 k-rows x 64 cols from X[k][col]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = tid + i * 256;
    int64_t r, c;
    if (KC) { r = r0 + idx / 8; c = k0 + (idx % 8) * 4; }
    else { r = k0 + idx / 16; c = r0 + (idx % 16) * 4; }
    const int64_t rlim = KC ? rows : kend, clim = KC ? kend : rows;
    if (VEC && r < rlim && c + 3 < clim) {
      const f32x4 x = *(const f32x4*)(X + r * ld + c);
#pragma unroll
      for (int u = 0; u < 4; ++u) v[i * 4 + u] = x[u];
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[i * 4 + u] = (r < rlim && c + u < clim) ? X[r * ld + c + u] : 0.0f;
    }
  }
}

template <bool KC>
__device__ __forceinline__ void store_op(float (*S)[kGLd], int tid, const float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = tid + i * 256;
    if (KC) {
      const int r = idx / 8, kq = (idx % 8) * 4;
#pragma unroll
      for (int u = 0; u < 4; ++u) S[kq + u][r] = v[i * 4 + u];
    } else {
      const int kr = idx / 16, c = (idx % 16) * 4;
      *(f32x4*)&S[kr][c] = f32x4{v[i * 4], v[i * 4 + 1], v[i * 4 + 2], v[i * 4 + 3]};
    }
  }
}

template <bool A_KC, bool B_KC, bool VEC>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* A, const float* B, float* C, int64_t m,
                                                       int64_t n, int64_t k, int64_t lda, int64_t ldb, int64_t ldc,
                                                       int64_t kchunk) {
  __shared__ __attribute__((aligned(16))) float As[kGBK][kGLd];
  __shared__ __attribute__((aligned(16))) float Bs[kGBK][kGLd];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.y * kGT, n0 = (int64_t)blockIdx.x * kGT;
  const int64_t kb = (int64_t)blockIdx.z * kchunk;
  const int64_t ke = kb + kchunk < k ? kb + kchunk : k;
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
  float va[8], vb[8];
  if (kb < ke) {
    load_op<A_KC, VEC>(A, lda, m0, m, kb, ke, tid, va);
    load_op<B_KC, VEC>(B, ldb, n0, n, kb, ke, tid, vb);
  }
  for (int64_t k0 = kb; k0 < ke; k0 += kGBK) {
    __syncthreads();
    store_op<A_KC>(As, tid, va);
    store_op<B_KC>(Bs, tid, vb);
    __syncthreads();
    if (k0 + kGBK < ke) {
      load_op<A_KC, VEC>(A, lda, m0, m, k0 + kGBK, ke, tid, va);
      load_op<B_KC, VEC>(B, ldb, n0, n, k0 + kGBK, ke, tid, vb);
    }
#pragma unroll
    for (int s = 0; s < kGBK / 2; ++s) {
      const float a = As[2 * s + h][wm * 32 + r];
      const float b = Bs[2 * s + h][wn * 32 + r];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
  }
  float* Cz = C + (int64_t)blockIdx.z * m * ldc;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int64_t row = m0 + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
    const int64_t col = n0 + wn * 32 + r;
    if (row < m && col < n) Cz[row * ldc + col] = acc[e];
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* ws, int64_t splits, int64_t m, int64_t n,
                                                            float* C, int64_t ldc) {
  const int64_t total = m * n;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    float s = ws[i];
    for (int64_t z = 1; z < splits; ++z) s += ws[z * total + i];
    const int64_t row = i / n, col = i % n;
    C[row * ldc + col] = s;
  }
}

__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float warp_add(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// one block (256 threads) per row: lse_i = log(sum exp(S_ij)); loss_i = lse_i - S_i,t
__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* S, int64_t m, int64_t n, int64_t tstride,
                                                     float* lse, float* row_loss) {
  __shared__ float red[4];
  const int64_t i = blockIdx.x;
  const float* row = S + i * n;
  float mx = -__builtin_inff();
  for (int64_t j = threadIdx.x; j < n; j += 256) mx = fmaxf(mx, row[j]);
  mx = warp_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int64_t j = threadIdx.x; j < n; j += 256) sum += expf(row[j] - mx);
  sum = warp_add(sum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float l = mx + logf(red[0] + red[1] + red[2] + red[3]);
    lse[i] = l;
    const int64_t t = i * tstride;
    row_loss[i] = l - row[t];
  }
}

// deterministic mean: one block sums the m row losses in a fixed order
__global__ __launch_bounds__(256) void mean_kernel(const float* v, int64_t m, float scale, float* out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t j = threadIdx.x; j < m; j += 256) s += v[j];
  s = warp_add(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = (red[0] + red[1] + red[2] + red[3]) / (float)m * scale;
}

__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* S, const float* lse, int64_t m, int64_t n,
                                                     int64_t tstride, const float* g, float scale, float* dS) {
  const int64_t i = blockIdx.x;
  const float coef = (g ? *g : 1.0f) * scale / (float)m;
  const float l = lse[i];
  const int64_t t = i * tstride;
  for (int64_t j = threadIdx.x; j < n; j += 256) {
    const float p = expf(S[i * n + j] - l);
    dS[i * n + j] = coef * (p - (j == t ? 1.0f : 0.0f));
  }
}

__global__ __launch_bounds__(256) void transpose_f32_kernel(const float* X, int64_t rows, int64_t cols, float* Y) {
  __shared__ float t[32][33];
  const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int yy = ty; yy < 32; yy += 8) {
    const int64_t r = r0 + yy, c = c0 + tx;
    t[yy][tx] = (r < rows && c < cols) ? X[r * cols + c] : 0.0f;
  }
  __syncthreads();
  for (int yy = ty; yy < 32; yy += 8) {
    const int64_t c = c0 + yy, r = r0 + tx;
    if (c < cols && r < rows) Y[c * rows + r] = t[tx][yy];
  }
}

}  // namespace drt

using namespace drt;

extern "C" {

int drt_gemm_nt_f32(const float* A, const float* B, float* C, int64_t m, int64_t n, int64_t k, int64_t lda,
                    int64_t ldb, int64_t ldc, void* stream) {
  DRT_REQUIRE(m >= 0 && n >= 0 && k >= 0 && lda >= k && ldb >= k && ldc >= n);
  if (m == 0 || n == 0) return DRT_OK;
  DRT_REQUIRE(C && (k == 0 || (A && B)));
  dim3 grid((unsigned)((n + kFT - 1) / kFT), (unsigned)((m + kFT - 1) / kFT));
  hipLaunchKernelGGL(gemm_nt_f32_kernel, grid, dim3(kF32Threads), 0, (hipStream_t)stream, A, B, C, m, n, k, lda,
                     ldb, ldc, 1.0f);
  return hip_status(hipGetLastError());
}

// C[m][n] = sum_k A(m,k) B(k,n); a_kc: A is [m][k] (else [k][m]); b_kc: B is [n][k] (else [k][n]).
// splits > 1: ws holds splits * m * n floats (deterministic split-K).
int drt_gemm_f32(const float* A, const float* B, float* C, int64_t m, int64_t n, int64_t k, int64_t lda,
                 int64_t ldb, int64_t ldc, int32_t a_kc, int32_t b_kc, int32_t splits, float* ws, void* stream) {
  DRT_REQUIRE(m >= 0 && n >= 0 && k >= 0 && ldc >= n && splits >= 1);
  DRT_REQUIRE(lda >= (a_kc ? k : m) && ldb >= (b_kc ? k : n));
  if (m == 0 || n == 0) return DRT_OK;
  DRT_REQUIRE(C && (k == 0 || (A && B)) && (splits == 1 || ws));
  hipStream_t s = (hipStream_t)stream;
  if (k == 0) return hip_status(hipMemset2DAsync(C, ldc * 4, 0, n * 4, m, s));
  int64_t kchunk = (k + splits - 1) / splits;
  kchunk = (kchunk + kGBK - 1) / kGBK * kGBK;
  const int64_t nz = (k + kchunk - 1) / kchunk;
  const bool vec = ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && lda % 4 == 0 && ldb % 4 == 0;
  float* out = nz > 1 ? ws : C;
  const int64_t ldo = nz > 1 ? n : ldc;
  dim3 grid((unsigned)((n + kGT - 1) / kGT), (unsigned)((m + kGT - 1) / kGT), (unsigned)nz);
#define GF32(AK, BK, V) hipLaunchKernelGGL((gemm_f32_kernel<AK, BK, V>), grid, dim3(256), 0, s, A, B, out, m, n, k, lda, ldb, ldo, kchunk)
  if (vec) {
    if (a_kc && b_kc) GF32(true, true, true);
    else if (a_kc) GF32(true, false, true);
    else if (b_kc) GF32(false, true, true);
    else GF32(false, false, true);
  } else {
    if (a_kc && b_kc) GF32(true, true, false);
    else if (a_kc) GF32(true, false, false);
    else if (b_kc) GF32(false, true, false);
    else GF32(false, false, false);
  }
#undef GF32
  if (nz > 1) {
    const int64_t blocks = (m * n + 255) / 256 < 2048 ? (m * n + 255) / 256 : 2048;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const float*)ws, nz, m, n, C,
                       ldc);
  }
  return hip_status(hipGetLastError());
}

int drt_ce_fwd(const float* S, int64_t m, int64_t n, int64_t target_stride, float scale, float* lse,
               float* row_loss, float* loss, void* stream) {
  DRT_REQUIRE(m > 0 && n > 0 && target_stride >= 0 && (m - 1) * target_stride < n);
  DRT_REQUIRE(S && lse && row_loss && loss);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_fwd_kernel, dim3((unsigned)m), dim3(256), 0, s, S, m, n, target_stride, lse, row_loss);
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(256), 0, s, (const float*)row_loss, m, scale, loss);
  return hip_status(hipGetLastError());
}

int drt_ce_bwd(const float* S, const float* lse, int64_t m, int64_t n, int64_t target_stride, const float* grad,
               float scale, float* dS, void* stream) {
  DRT_REQUIRE(m > 0 && n > 0 && target_stride >= 0 && (m - 1) * target_stride < n);
  DRT_REQUIRE(S && lse && dS);
  hipLaunchKernelGGL(ce_bwd_kernel, dim3((unsigned)m), dim3(256), 0, (hipStream_t)stream, S, lse, m, n,
                     target_stride, grad, scale, dS);
  return hip_status(hipGetLastError());
}

int drt_transpose_f32(const float* X, int64_t rows, int64_t cols, float* Y, void* stream) {
  DRT_REQUIRE(rows >= 0 && cols >= 0);
  if (rows == 0 || cols == 0) return DRT_OK;
  DRT_REQUIRE(X && Y);
  dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32));
  hipLaunchKernelGGL(transpose_f32_kernel, grid, dim3(256), 0, (hipStream_t)stream, X, rows, cols, Y);
  return hip_status(hipGetLastError());
}

}  // extern "C"
