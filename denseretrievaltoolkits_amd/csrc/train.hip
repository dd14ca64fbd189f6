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

// One 64 x 64 output tile (tile_m, tile_n) over k in [kz * kchunk, ...) into C + kz * m * ldc.
template <bool A_KC, bool B_KC, bool VEC>
__device__ __forceinline__ void gemm_f32_tile(const float* A, const float* B, float* C, int64_t m, int64_t n,
                                              int64_t k, int64_t lda, int64_t ldb, int64_t ldc, int64_t kchunk,
                                              int64_t tile_m, int64_t tile_n, int64_t kz,
                                              float (*As)[kGLd], float (*Bs)[kGLd]) {
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = tile_m * kGT, n0 = tile_n * kGT;
  const int64_t kb = kz * kchunk;
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
  float* Cz = C + kz * m * ldc;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int64_t row = m0 + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
    const int64_t col = n0 + wn * 32 + r;
    if (row < m && col < n) Cz[row * ldc + col] = acc[e];
  }
}

template <bool A_KC, bool B_KC, bool VEC>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* A, const float* B, float* C, int64_t m,
                                                       int64_t n, int64_t k, int64_t lda, int64_t ldb, int64_t ldc,
                                                       int64_t kchunk) {
  __shared__ __attribute__((aligned(16))) float As[kGBK][kGLd];
  __shared__ __attribute__((aligned(16))) float Bs[kGBK][kGLd];
  gemm_f32_tile<A_KC, B_KC, VEC>(A, B, C, m, n, k, lda, ldb, ldc, kchunk, blockIdx.y, blockIdx.x, blockIdx.z, As, Bs);
}

// Score-matrix backward, both GEMMs in ONE launch (split-K partials into ws):
//   problem 0: dq [m][d] = dS [m][n] . p [n][d]       (A k-contiguous, B [k][n])
//   problem 1: dp [n][d] = dS^T   . q [m][d]          (A = dS read as [k][m], B [k][n])
// block b < t0 * z0 -> problem 0, else problem 1; z = split index.
struct DualGemm {
  const float* dS; const float* p; const float* q;
  float* ws0; float* ws1;
  int64_t m, n, d;
  int64_t kchunk0, kchunk1, z0, z1, tn;   // tn = d tiles
};

template <bool VEC>
__global__ __launch_bounds__(256) void gemm_f32_dual_kernel(DualGemm g) {
  __shared__ __attribute__((aligned(16))) float As[kGBK][kGLd];
  __shared__ __attribute__((aligned(16))) float Bs[kGBK][kGLd];
  int64_t b = blockIdx.x;
  const int64_t tm0 = (g.m + kGT - 1) / kGT;
  const int64_t nb0 = tm0 * g.tn * g.z0;
  if (b < nb0) {
    const int64_t kz = b / (tm0 * g.tn), t = b % (tm0 * g.tn);
    gemm_f32_tile<true, false, VEC>(g.dS, g.p, g.ws0, g.m, g.d, g.n, g.n, g.d, g.d, g.kchunk0, t / g.tn, t % g.tn,
                                     kz, As, Bs);
  } else {
    b -= nb0;
    const int64_t tm1 = (g.n + kGT - 1) / kGT;
    const int64_t kz = b / (tm1 * g.tn), t = b % (tm1 * g.tn);
    gemm_f32_tile<false, false, VEC>(g.dS, g.q, g.ws1, g.n, g.d, g.m, g.n, g.d, g.d, g.kchunk1, t / g.tn,
                                      t % g.tn, kz, As, Bs);
  }
}

// Fixed-order split-K sums of both problems: out0 [m0 x d] from z0 partials, out1 [m1 x d] from z1.
__global__ __launch_bounds__(256) void dual_reduce_kernel(const float* ws0, int64_t z0, int64_t e0, float* out0,
                                                          const float* ws1, int64_t z1, int64_t e1, float* out1) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < e0 + e1; i += (int64_t)gridDim.x * 256) {
    const bool first = i < e0;
    const int64_t j = first ? i : i - e0;
    const float* w = first ? ws0 : ws1;
    const int64_t z = first ? z0 : z1, e = first ? e0 : e1;
    float s = w[j];
    for (int64_t u = 1; u < z; ++u) s += w[u * e + j];
    (first ? out0 : out1)[j] = s;
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

// ---------------------------------------------------------------------------
// Large-tile exact-f32 GEMM (round 6, the score matrix and its backward at the C3 shape).
// The 64 x 64 kernel above moves 1/16 B of operands per flop through VGPR staging and
// ds_write_b32 between two barriers per K-step; at 512 x 4096 x 768 it runs at 0.53 of the
// f32 MFMA rate.  Here a TM x TN block (TM = 128; TN = 64 forward, 96 backward) lands its
// 32-deep K-steps global -> LDS with global_load_lds_dwordx4 in a STAGES-slot ring (no
// staging registers, no LDS stores, one barrier per step) and each wave runs MT x NT
// v_mfma_f32_32x32x2_f32 tiles.
//   k-contiguous operand (q, p, dS as [m][n]): image [rows][8 x 16 B], chunk c of row r at
//     position c ^ ((r >> 1) & 7); in a K-step lane (r, h) carries k = 16 h + s at MFMA s, so it
//     reads its 16 k as 4 ds_read_b128 (conflict-free for every b128 lane group with this XOR).
//   k-major operand (p / q as [k][d], dS^T): image [32 k][cols] fp32 as stored; lane (c, h)
//     reads k row 16 h + s with one ds_read_b32 (32 consecutive floats per lane group).
// The k order inside a step differs from the 64 x 64 kernel's (both are exact-f32 fmaf
// chains; results agree to f32 rounding).  Blocks are remapped so that an XCD's blocks are
// contiguous tiles sharing an operand panel (the wide operand is read into each L2 once).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void f32_glds16(const void* gsrc, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}

__device__ __forceinline__ uint32_t f32_lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

struct F32Prob {
  const float* A;   // KC: [m][lda] (row i, k) ; else [k][lda] (k, row i)
  const float* B;   // KC: [n][ldb] ; else [k][ldb]
  float* C;         // [m][ldc]; split z writes C + z * m * ldc
  int64_t m, n, k, lda, ldb, ldc;
  int64_t kchunk;   // k per split, multiple of 32
  int tiles_m, tiles_n, splits;
  int m_fast;       // block order inside the problem: 1 = m-tiles of one n-panel adjacent
};

// One operand's 32-deep K-step (ROWS rows of the output side) into its ring slot.  KC: 1 KiB
// wave-instruction J = rows 8J .. 8J + 7 (rows past `rows` clamped: masked outputs); k-major:
// J = floats [256 J, 256 J + 256) of the [32][ROWS] image (columns past `rows` clamped; `rows`
// % 4 == 0 keeps every 16-B chunk whole).
template <int ROWS, bool KC>
__device__ __forceinline__ void f32_stage(const float* X, int64_t ld, int64_t r0, int64_t rows, int64_t k0,
                                          uint32_t lds, int wave, int lane) {
  constexpr int NI = ROWS / 8;
  static_assert(NI % 4 == 0, "4 waves share the wave-instructions");
#pragma unroll
  for (int J0 = 0; J0 < NI; J0 += 4) {
    const int J = J0 + wave;
    const float* p;
    if (KC) {
      const int row = 8 * J + (lane >> 3);
      int64_t gr = r0 + row;
      gr = gr < rows ? gr : rows - 1;
      const int chunk = (lane & 7) ^ ((4 * J + (lane >> 4)) & 7);
      p = X + gr * ld + k0 + chunk * 4;
    } else {
      const int f = J * 256 + lane * 4;
      const int kr = f / ROWS, col = f - kr * ROWS;
      int64_t gc = r0 + col;
      gc = gc < rows ? gc : rows - 4;
      p = X + (k0 + kr) * ld + gc;
    }
    f32_glds16(p, __builtin_amdgcn_readfirstlane(lds + J * 1024));
  }
}

// s_waitcnt vmcnt(PER * n): all but the n youngest K-steps (PER LDS-DMA per wave each) landed.
template <int PER>
__device__ __forceinline__ void f32_wait_steps(int n) {
  if (n <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
}

template <int TM, int TN, int WM, int WN, bool A_KC, bool B_KC, int STAGES>
struct F32Cfg {
  static constexpr int kA = TM * 128, kB = TN * 128, kStage = kA + kB, kLds = STAGES * kStage;
  static constexpr int kPer = kStage / 4096;            // LDS-DMA per wave per K-step
  static constexpr int MT = TM / WM / 32, NT = TN / WN / 32;
  static_assert(WM * WN == 4 && MT * WM * 32 == TM && NT * WN * 32 == TN, "4 waves of 32 x 32 tiles");
  static_assert(STAGES >= 2 && STAGES <= 4, "ring depth");
};

template <int TM, int TN, int WM, int WN, bool A_KC, bool B_KC, int STAGES>
__device__ __forceinline__ void f32x_block(const F32Prob& g, int64_t wg, char* smem) {
  using Cfg = F32Cfg<TM, TN, WM, WN, A_KC, B_KC, STAGES>;
  constexpr int MT = Cfg::MT, NT = Cfg::NT;
  const int per_split = g.tiles_m * g.tiles_n;
  const int z = (int)(wg / per_split);
  const int t = (int)(wg - (int64_t)z * per_split);
  const int tm = g.m_fast ? t % g.tiles_m : t / g.tiles_n;
  const int tn = g.m_fast ? t / g.tiles_m : t % g.tiles_n;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave / WN, wn = wave % WN;
  const int64_t m0 = (int64_t)tm * TM, n0 = (int64_t)tn * TN;
  const int64_t kb = (int64_t)z * g.kchunk;
  const int64_t ke = kb + g.kchunk < g.k ? kb + g.kchunk : g.k;
  const int nt = (int)((ke - kb) / 32);
  const uint32_t lds0 = f32_lds_addr(smem);
  auto stage = [&](int s, int slot) {
    const uint32_t base = lds0 + slot * Cfg::kStage;
    f32_stage<TM, A_KC>(g.A, g.lda, m0, g.m, kb + (int64_t)s * 32, base, wave, lane);
    f32_stage<TN, B_KC>(g.B, g.ldb, n0, g.n, kb + (int64_t)s * 32, base + Cfg::kA, wave, lane);
  };
  f32x16 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nt) stage(s, s);
  // per-lane read offsets: KC rows r of each 32-row tile (XOR (r >> 1) & 7), k-major column r, k row 16 h
  const int swz = (r >> 1) & 7;
  const int arow = wm * MT * 32 + r, brow = wn * NT * 32 + r;
  for (int s = 0; s < nt; ++s) {
    const int younger = nt - 1 - s < STAGES - 2 ? nt - 1 - s : STAGES - 2;
    f32_wait_steps<Cfg::kPer>(younger);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (s + STAGES - 1 < nt) stage(s + STAGES - 1, (s + STAGES - 1) % STAGES);
    const char* As = smem + (s % STAGES) * Cfg::kStage;
    const char* Bs = As + Cfg::kA;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 av[MT], bv[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if (A_KC) {
          av[i] = *(const f32x4*)(As + (arow + i * 32) * 128 + (((4 * h + j) ^ swz) << 4));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) av[i][e] = ((const float*)As)[(16 * h + 4 * j + e) * TM + arow + i * 32];
        }
      }
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        if (B_KC) {
          bv[i] = *(const f32x4*)(Bs + (brow + i * 32) * 128 + (((4 * h + j) ^ swz) << 4));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) bv[i][e] = ((const float*)Bs)[(16 * h + 4 * j + e) * TN + brow + i * 32];
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int jj = 0; jj < NT; ++jj)
            acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][e], bv[jj][e], acc[i][jj], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  float* Cz = g.C + (int64_t)z * g.m * g.ldc;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int jj = 0; jj < NT; ++jj)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t row = m0 + wm * MT * 32 + i * 32 + 8 * (e >> 2) + 4 * h + (e & 3);
        const int64_t col = n0 + wn * NT * 32 + jj * 32 + r;
        if (row < g.m && col < g.n) Cz[row * g.ldc + col] = acc[i][jj][e];
      }
}

// XCD-contiguous block rank (blocks b, b + 8, ... run on XCD b % 8): an XCD's blocks are a
// contiguous range of the problem's (split, tile) order.
__device__ __forceinline__ int64_t f32_xcd_rank(int64_t bid, int64_t nwg) {
  const int64_t xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

// forward: S (or split partials) = q . p^T, both k-contiguous
constexpr int kFwdTN = 64, kFwdStages = 4;
using FwdCfg = F32Cfg<128, kFwdTN, 2, 2, true, true, kFwdStages>;
__global__ __launch_bounds__(256) void score_fwd_gemm_kernel(F32Prob g) {
  __shared__ __attribute__((aligned(16))) char smem[FwdCfg::kLds];
  f32x_block<128, kFwdTN, 2, 2, true, true, kFwdStages>(g, f32_xcd_rank(blockIdx.x, gridDim.x), smem);
}

// backward, both GEMMs in one grid: problem 0 dq = dS . p (dS k-contiguous, p k-major),
// problem 1 dp = dS^T . q (both k-major); blocks [0, nb0) are problem 0.
constexpr int kBwdTN = 96, kBwdStages = 2;
using Bwd0Cfg = F32Cfg<128, kBwdTN, 4, 1, true, false, kBwdStages>;
using Bwd1Cfg = F32Cfg<128, kBwdTN, 4, 1, false, false, kBwdStages>;
static_assert(Bwd0Cfg::kLds == Bwd1Cfg::kLds, "one LDS size");
__global__ __launch_bounds__(256) void score_bwd_gemm_kernel(F32Prob g0, F32Prob g1, int64_t nb0) {
  __shared__ __attribute__((aligned(16))) char smem[Bwd0Cfg::kLds];
  const int64_t wg = f32_xcd_rank(blockIdx.x, gridDim.x);
  if (wg < nb0) f32x_block<128, kBwdTN, 4, 1, true, false, kBwdStages>(g0, wg, smem);
  else f32x_block<128, kBwdTN, 4, 1, false, false, kBwdStages>(g1, wg - nb0, smem);
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

// Forward row pass fused with the split-K reduction: row i of S = sum of the z partials
// (fixed order), written out, then lse_i and loss_i as ce_fwd_kernel.
__global__ __launch_bounds__(256) void ce_fwd_reduce_kernel(const float* ws, int64_t z, float* S, int64_t m,
                                                            int64_t n, int64_t tstride, float* lse, float* row_loss) {
  __shared__ float red[4];
  __shared__ float target_score;
  const int64_t i = blockIdx.x;
  float* row = S + i * n;
  const int64_t e = m * n, t = i * tstride;
  float mx = -__builtin_inff();
  for (int64_t j = threadIdx.x; j < n; j += 256) {
    float v = ws[i * n + j];
    for (int64_t u = 1; u < z; ++u) v += ws[u * e + i * n + j];
    row[j] = v;
    if (j == t) target_score = v;
    mx = fmaxf(mx, v);
  }
  mx = warp_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int64_t j = threadIdx.x; j < n; j += 256) sum += expf(row[j] - mx);   // own writes: same thread
  sum = warp_add(sum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float l = mx + logf(red[0] + red[1] + red[2] + red[3]);
    lse[i] = l;
    row_loss[i] = l - target_score;
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

// ---- fused score + CE (one host call per direction; workspace from drt_score_ce_workspace)
static void split_plan(int64_t m, int64_t n, int64_t k, int64_t& kchunk, int64_t& nz) {
  // split K until ~320 blocks of 64 x 64 tiles are in flight (>= 128 k per split)
  const int64_t tiles = ((m + kGT - 1) / kGT) * ((n + kGT - 1) / kGT);
  int64_t splits = (320 + tiles - 1) / tiles;
  if (splits > k / 128) splits = k / 128;
  if (splits < 1) splits = 1;
  kchunk = (k + splits - 1) / splits;
  kchunk = (kchunk + kGBK - 1) / kGBK * kGBK;
  nz = k > 0 ? (k + kchunk - 1) / kchunk : 1;
}

static int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Large-tile path: every K range whole 32-deep steps (m, n, d multiples of 32), 16-B aligned rows.
static bool large_f32_shape(int64_t m, int64_t n, int64_t d) { return m % 32 == 0 && n % 32 == 0 && d % 32 == 0; }
static bool large_f32_ok(const float* q, const float* p, int64_t m, int64_t n, int64_t d) {
  return large_f32_shape(m, n, d) && (uintptr_t)q % 16 == 0 && (uintptr_t)p % 16 == 0;
}

// forward: 128 x 64 tiles, K split until ~256 blocks (one per CU; >= 2 steps per split)
static void fwd_plan_large(int64_t m, int64_t n, int64_t d, int64_t& kc, int64_t& z) {
  const int64_t tiles = cdiv(m, 128) * cdiv(n, kFwdTN);
  int64_t splits = cdiv(256, tiles);
  if (splits > d / 64) splits = d / 64;
  if (splits < 1) splits = 1;
  kc = cdiv(cdiv(d, splits), 32) * 32;
  z = cdiv(d, kc);
}

// backward: 128 x 96 tiles of dq [m][d] (K = n) and dp [n][d] (K = m), one K chunk for both so every
// block carries the same work, sized for ~512 blocks (two per CU); a problem whose K fits one chunk
// writes its output directly.
static void bwd_plan_large(int64_t m, int64_t n, int64_t d, int64_t& kc0, int64_t& z0, int64_t& kc1, int64_t& z1) {
  const int64_t tn = cdiv(d, kBwdTN);
  const int64_t work = cdiv(m, 128) * tn * n + cdiv(n, 128) * tn * m;
  int64_t kc = cdiv(cdiv(work, 512), 32) * 32;
  if (kc < 128) kc = 128;
  kc0 = kc < n ? kc : n;
  z0 = cdiv(n, kc0);
  kc1 = kc < m ? kc : m;
  z1 = cdiv(m, kc1);
}

static size_t score_ce_ws_floats(int64_t m, int64_t n, int64_t d, size_t* fwd, size_t* bwd) {
  int64_t kc, z, kc0, z0, kc1, z1;
  split_plan(m, n, d, kc, z);
  split_plan(m, d, n, kc0, z0);
  split_plan(n, d, m, kc1, z1);
  size_t f = (size_t)z * m * n + (size_t)m;
  size_t b = (size_t)m * n + (size_t)z0 * m * d + (size_t)z1 * n * d;
  if (large_f32_shape(m, n, d)) {   // the large-tile plan may split differently: room for either
    fwd_plan_large(m, n, d, kc, z);
    bwd_plan_large(m, n, d, kc0, z0, kc1, z1);
    const size_t fl = (z > 1 ? (size_t)z * m * n : 0) + (size_t)m;
    const size_t bl = (size_t)m * n + (z0 > 1 ? (size_t)z0 * m * d : 0) + (z1 > 1 ? (size_t)z1 * n * d : 0);
    f = f > fl ? f : fl;
    b = b > bl ? b : bl;
  }
  if (fwd) *fwd = f;
  if (bwd) *bwd = b;
  return f > b ? f : b;
}

size_t drt_score_ce_workspace(int64_t m, int64_t n, int32_t d) {
  if (m <= 0 || n <= 0 || d <= 0) return 0;
  return score_ce_ws_floats(m, n, d, nullptr, nullptr) * sizeof(float);
}

// S = q . p^T (exact f32), lse, loss = scale * mean_i (lse_i - S[i][i * target_stride]).
// 3 launches: GEMM (split-K partials or S itself) -> per-row (split reduce + LSE + row loss) ->
// fixed-order mean.
int drt_score_ce_fwd(const float* q, const float* p, int64_t m, int64_t n, int32_t d, int64_t target_stride,
                     float scale, float* S, float* lse, float* loss, void* ws, size_t ws_bytes, void* stream) {
  DRT_REQUIRE(m > 0 && n > 0 && d > 0 && target_stride >= 0 && (m - 1) * target_stride < n);
  DRT_REQUIRE(q && p && S && lse && loss && ws && ws_bytes >= drt_score_ce_workspace(m, n, d));
  hipStream_t s = (hipStream_t)stream;
  int64_t kc, z;
  float* part = (float*)ws;
  if (large_f32_ok(q, p, m, n, d)) {
    fwd_plan_large(m, n, d, kc, z);
    float* row_loss = part + (z > 1 ? (size_t)z * m * n : 0);
    F32Prob g{q, p, z > 1 ? part : S, m, n, (int64_t)d, (int64_t)d, (int64_t)d, n, kc,
              (int)cdiv(m, 128), (int)cdiv(n, kFwdTN), (int)z, 1};
    const int64_t blocks = (int64_t)g.tiles_m * g.tiles_n * z;
    hipLaunchKernelGGL(score_fwd_gemm_kernel, dim3((unsigned)blocks), dim3(256), 0, s, g);
    if (z > 1)
      hipLaunchKernelGGL(ce_fwd_reduce_kernel, dim3((unsigned)m), dim3(256), 0, s, (const float*)part, z, S, m, n,
                         target_stride, lse, row_loss);
    else
      hipLaunchKernelGGL(ce_fwd_kernel, dim3((unsigned)m), dim3(256), 0, s, (const float*)S, m, n, target_stride,
                         lse, row_loss);
    hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(256), 0, s, (const float*)row_loss, m, scale, loss);
    return hip_status(hipGetLastError());
  }
  split_plan(m, n, d, kc, z);
  float* row_loss = part + (size_t)z * m * n;
  const bool vec = ((uintptr_t)q % 16 == 0) && ((uintptr_t)p % 16 == 0) && d % 4 == 0;
  dim3 grid((unsigned)((n + kGT - 1) / kGT), (unsigned)((m + kGT - 1) / kGT), (unsigned)z);
  if (vec) hipLaunchKernelGGL((gemm_f32_kernel<true, true, true>), grid, dim3(256), 0, s, q, p, part, m, n,
                              (int64_t)d, (int64_t)d, (int64_t)d, n, kc);
  else hipLaunchKernelGGL((gemm_f32_kernel<true, true, false>), grid, dim3(256), 0, s, q, p, part, m, n,
                          (int64_t)d, (int64_t)d, (int64_t)d, n, kc);
  hipLaunchKernelGGL(ce_fwd_reduce_kernel, dim3((unsigned)m), dim3(256), 0, s, (const float*)part, z, S, m, n,
                     target_stride, lse, row_loss);
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(256), 0, s, (const float*)row_loss, m, scale, loss);
  return hip_status(hipGetLastError());
}

// dS = scale * g / m * (softmax(S) - onehot); dq = dS . p; dp = dS^T . q.
// 3 launches: dS -> both GEMMs in one grid (split-K partials) -> both fixed-order reductions.
int drt_score_ce_bwd(const float* q, const float* p, const float* S, const float* lse, int64_t m, int64_t n,
                     int32_t d, int64_t target_stride, const float* grad, float scale, float* dq, float* dp,
                     void* ws, size_t ws_bytes, void* stream) {
  DRT_REQUIRE(m > 0 && n > 0 && d > 0 && target_stride >= 0 && (m - 1) * target_stride < n);
  DRT_REQUIRE(q && p && S && lse && dq && dp && ws && ws_bytes >= drt_score_ce_workspace(m, n, d));
  hipStream_t s = (hipStream_t)stream;
  float* dS = (float*)ws;
  int64_t kc0, z0, kc1, z1;
  if (large_f32_ok(q, p, m, n, d)) {
    bwd_plan_large(m, n, d, kc0, z0, kc1, z1);
    float* ws0 = dS + (size_t)m * n;
    float* ws1 = ws0 + (z0 > 1 ? (size_t)z0 * m * d : 0);
    const int tn = (int)cdiv(d, kBwdTN);
    F32Prob g0{dS, p, z0 > 1 ? ws0 : dq, m, (int64_t)d, n, n, (int64_t)d, (int64_t)d, kc0,
               (int)cdiv(m, 128), tn, (int)z0, 0};
    F32Prob g1{dS, q, z1 > 1 ? ws1 : dp, n, (int64_t)d, m, n, (int64_t)d, (int64_t)d, kc1,
               (int)cdiv(n, 128), tn, (int)z1, 0};
    const int64_t nb0 = (int64_t)g0.tiles_m * tn * z0, nb1 = (int64_t)g1.tiles_m * tn * z1;
    hipLaunchKernelGGL(ce_bwd_kernel, dim3((unsigned)m), dim3(256), 0, s, S, lse, m, n, target_stride, grad, scale,
                       dS);
    hipLaunchKernelGGL(score_bwd_gemm_kernel, dim3((unsigned)(nb0 + nb1)), dim3(256), 0, s, g0, g1, nb0);
    const int64_t e0 = z0 > 1 ? m * d : 0, e1 = z1 > 1 ? n * d : 0;
    if (e0 + e1 > 0) {
      const int64_t rb = (e0 + e1 + 255) / 256 < 2048 ? (e0 + e1 + 255) / 256 : 2048;
      hipLaunchKernelGGL(dual_reduce_kernel, dim3((unsigned)rb), dim3(256), 0, s, (const float*)ws0, z0, e0, dq,
                         (const float*)ws1, z1, e1, dp);
    }
    return hip_status(hipGetLastError());
  }
  DualGemm g{};
  split_plan(m, d, n, kc0, z0);
  split_plan(n, d, m, kc1, z1);
  g.dS = dS; g.p = p; g.q = q;
  g.ws0 = dS + (size_t)m * n;
  g.ws1 = g.ws0 + (size_t)z0 * m * d;
  g.m = m; g.n = n; g.d = d;
  g.kchunk0 = kc0; g.kchunk1 = kc1; g.z0 = z0; g.z1 = z1;
  g.tn = (d + kGT - 1) / kGT;
  hipLaunchKernelGGL(ce_bwd_kernel, dim3((unsigned)m), dim3(256), 0, s, S, lse, m, n, target_stride, grad, scale, dS);
  const int64_t blocks = ((m + kGT - 1) / kGT) * g.tn * z0 + ((n + kGT - 1) / kGT) * g.tn * z1;
  const bool vec = ((uintptr_t)q % 16 == 0) && ((uintptr_t)p % 16 == 0) && d % 4 == 0 && n % 4 == 0;
  if (vec) hipLaunchKernelGGL(gemm_f32_dual_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, g);
  else hipLaunchKernelGGL(gemm_f32_dual_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, g);
  const int64_t e0 = m * d, e1 = n * d;
  const int64_t rb = (e0 + e1 + 255) / 256 < 2048 ? (e0 + e1 + 255) / 256 : 2048;
  hipLaunchKernelGGL(dual_reduce_kernel, dim3((unsigned)rb), dim3(256), 0, s, (const float*)g.ws0, z0, e0, dq,
                     (const float*)g.ws1, z1, e1, dp);
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
