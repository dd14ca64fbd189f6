// NT GEMM on CDNA4 MFMA:  C[m, n] = sum_k A[m, k] * B[n, k]  (+ epilogue)
//
// Both operands are K-contiguous ("x @ W^T" with an nn.Linear weight [out, in],
// and q_reps @ p_reps^T for the in-batch score matrix,
// DRT/model/biencoder.py:107 / DRT/trainer/losses.py:16), so one kernel shape
// serves the encoder projections and the training scores.
//
// Tile 128 x 128 x 64, 4 waves (2 x 2), each wave 64 x 64 = 2 x 2 tiles of
// v_mfma_f32_32x32x16_bf16.  A and B tiles are staged global -> LDS with
// global_load_lds_dwordx4 (inline asm, counted vmcnt), 2-slot ring, in the
// same XOR-swizzled [row][8 x 16 B] image as the search scan so the
// ds_read_b128 fragment reads are bank-conflict free.
#include "drt_common.h"
#include "ln_row.h"
#include "profile.h"

namespace drt {

constexpr int kGemmThreads = 256;
constexpr int kBM = 128, kBN = 128, kBK = 64;
constexpr int kTileA = kBM * kBK * 2;  // 16 KiB
constexpr int kTileB = kBN * kBK * 2;  // 16 KiB
constexpr int kStage = kTileA + kTileB;
constexpr int kGemmLds = 2 * kStage;   // 64 KiB -> 2 work-groups per CU
constexpr int kL = 256;                // 256^2 kernels: tile edge
constexpr int kLThreads = 512;

struct GemmArgs {
  const __bf16* A;   // [m][lda]
  const __bf16* B;   // [n][ldb]
  void* C;           // [m][ldc]  fp32 or bf16
  const float* bias; // [n] or null
  const __bf16* R;   // residual [m][ldr] or null
  int64_t m, n, k;
  int64_t lda, ldb, ldc, ldr;
  float alpha;
  int order;                // tile order within an XCD's range (tile_order)
  int64_t kchunk;           // split-K (128^2 kernel, PART): k per split; ws [splits][m][n] fp32
  float* ws;
  void* C2;                 // EPI_PRE: bf16 [m][ldc] pre-activation (bias added, before GELU)
  float drop_p;             // EPI_DROP: dropout probability, hash seed and site (drt_common.h)
  uint64_t seed, site;
  float* csum;              // optional (whole-line kernel, fp32-staged epilogue): column sums of the
                            // stored output per 128-row half tile, [2 * ceil(m / 256)][n]
};

__device__ __forceinline__ void g_glds16(const void* gsrc, uint32_t lds_addr) {
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

__device__ __forceinline__ uint32_t g_lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// Stage a 128-row x 64-col bf16 panel: 16 wave-instructions of 8 rows x 128 B,
// 4 per wave.  Rows past `rows` are clamped (masked in the epilogue).
__device__ __forceinline__ void stage_panel(const __bf16* base, int64_t ld, int64_t row0, int64_t rows,
                                            int64_t k0, uint32_t lds, int wave, int lane) {
  const int rsub = lane >> 3, pos = lane & 7;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int J = j * 4 + wave;           // 0..15
    const int row = J * 8 + rsub;         // 0..127
    int64_t gr = row0 + row;
    gr = gr < rows ? gr : rows - 1;
    const int c = pos ^ ((row >> 1) & 7);
    g_glds16(base + gr * ld + k0 + c * 8, __builtin_amdgcn_readfirstlane(lds + J * 1024));
  }
}

__device__ __forceinline__ float gelu_erf(float x) {
  // transformers ACT2FN["gelu"] = GELUActivation: x * 0.5 * (1 + erf(x / sqrt(2)))
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}

// GELU(erf) with erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below
// the bf16 rounding of the stored activation): one rcp, one exp, 6 FMA.
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);
  const float erf_abs = fmaf(-p, e, 1.0f);
  const float erf_v = x < 0.f ? -erf_abs : erf_abs;
  return 0.5f * x * (1.0f + erf_v);
}

// gelu_fast on two elements with packed fp32 math (v_pk_mul_f32 / v_pk_fma_f32: half the
// VALU issue of two scalar calls; the transcendentals stay per element).  The same A&S
// polynomial; 0.5 x (1 + sign(x) erf|.|) is evaluated as 0.5 x + 0.5 |x| erf|.| (one fma).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_fast2(f32x2 x) {
  f32x2 z = {fabsf(x.x), fabsf(x.y)};
  z = z * 0.70710678118654752f;
  const f32x2 d = z * 0.3275911f + 1.0f;
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = t * 1.061405429f - 1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t - 0.284496736f;
  p = p * t + 0.254829592f;
  p = p * t;
  const f32x2 ar = -(z * z) * 1.4426950408889634f;
  const f32x2 e = {__builtin_amdgcn_exp2f(ar.x), __builtin_amdgcn_exp2f(ar.y)};
  const f32x2 ea = 1.0f - p * e;
  const f32x2 hx = x * 0.5f;
  const f32x2 ha = {fabsf(hx.x), fabsf(hx.y)};
  return hx + ha * ea;
}

// EPI_DGELU: multiply by GELU'(R) (the dgrad of a GELU input: R = the bf16 pre-activation);
// EPI_PRE: also store the pre-activation to C2 (the training forward keeps it for the backward);
// EPI_DROP: dropout (counter hash of the flat output index, the mask drt_dropout_add_bf16 draws)
// applied after bias / GELU, before the residual.
enum { EPI_NONE = 0, EPI_BIAS = 1, EPI_GELU = 2, EPI_RESID = 4, EPI_DGELU = 8, EPI_PRE = 16, EPI_DROP = 32 };
constexpr int EPI_AUX = EPI_RESID | EPI_DGELU;   // epilogues that read R

// d/dx [x Phi(x)] = Phi(x) + x phi(x), erf by Abramowitz & Stegun 7.1.26 as gelu_fast
// (phi shares gelu_fast's exp(-x^2 / 2)).
__device__ __forceinline__ float gelu_grad(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);
  const float erf_abs = fmaf(-p, e, 1.0f);
  const float erf_v = x < 0.f ? -erf_abs : erf_abs;
  return fmaf(x * 0.39894228040143268f, e, 0.5f * (1.0f + erf_v));
}

// The part of the epilogue after bias / GELU, element (row, col): dropout, residual, GELU'.
template <int EPI>
__device__ __forceinline__ float epi_post(const GemmArgs& a, float v, int64_t row, int64_t col, float aux) {
  if (EPI & EPI_DROP) {
    const bool keep = drop_hash24(a.seed, a.site, (uint64_t)(row * a.ldc + col)) >= drop_threshold(a.drop_p);
    v = keep ? v * (1.0f / (1.0f - a.drop_p)) : 0.0f;
  }
  if (EPI & EPI_RESID) v += aux;
  if (EPI & EPI_DGELU) v *= gelu_grad(aux);
  return v;
}

// 256^2 kernel from this many 256^2 tiles up (tools/qsweep.py: 128 beats 512 by 16-22 % on 4k-16k-token
// batches); tile order inside an XCD's range: grouped-8 for K <= 1024 (small panels), row-major otherwise
// (profiles/r02o_gemm_tile_order.log: orders within noise).
constexpr int64_t kLargeMinTiles = 128;
__host__ __device__ constexpr int auto_tile_order(int64_t k) { return k <= 1024 ? 1 : 0; }

// NS = LDS stages of 32 KiB (A + B K-tile): 2 = double buffer, 2 work-groups per CU (grids of
// more than one round); 4 = a ring with two K-tiles in flight across each barrier (counted vmcnt,
// raw s_barrier), one work-group per CU -- for grids of at most one round (query-sized batches),
// where the double buffer's one-K-tile prefetch left every K-step waiting on an L2 round trip.
template <bool OUT_BF16, int EPI, bool PART = false, int NS = 2>
__global__ __launch_bounds__(kGemmThreads, NS == 2 ? 2 : 1) void gemm_nt_kernel(GemmArgs a) {
  static_assert(NS == 2 || NS == 4, "stage counts with vmcnt immediates below");
  __shared__ __attribute__((aligned(16))) char smem[NS * kStage];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap: blocks b and b+8 share an XCD (and its L2),
  // so give each XCD a contiguous run of tiles along n (shared A panel).
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tiles_n = (int)((a.n + kBN - 1) / kBN);
  const int64_t m0 = (int64_t)(wg / tiles_n) * kBM;
  const int64_t n0 = (int64_t)(wg % tiles_n) * kBN;

  const uint32_t lds0 = g_lds_addr(smem);
  // PART: this block sums k in [kbeg, kend) of split blockIdx.z (kchunk % kBK == 0)
  const int64_t kbeg = PART ? (int64_t)blockIdx.z * a.kchunk : 0;
  const int64_t kend = PART ? (kbeg + a.kchunk < a.k ? kbeg + a.kchunk : a.k) : a.k;
  const int ksteps = (int)((kend - kbeg) / kBK);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  const int sw = (r >> 1) & 7;
  int aoff[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) aoff[s] = r * 128 + ((((2 * s) | h) ^ sw) << 4);

  // one K-tile = 8 LDS-DMA wave-instructions per wave (4 of A, 4 of B)
  auto stage_k = [&](int kt, int slot) {
    const uint32_t nb = lds0 + slot * kStage;
    stage_panel(a.A, a.lda, m0, a.m, kbeg + (int64_t)kt * kBK, nb, wave, lane);
    stage_panel(a.B, a.ldb, n0, a.n, kbeg + (int64_t)kt * kBK, nb + kTileA, wave, lane);
  };
#pragma unroll
  for (int st = 0; st < NS - 1; ++st)
    if (st < ksteps) stage_k(st, st);

  int slot = 0;
  for (int kt = 0; kt < ksteps; ++kt) {
    if (NS == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {   // K-tile kt landed; the (at most NS - 2) tiles issued after it may stay in flight
      const int after = ksteps - 1 - kt;
      if (after >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if (after == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // WAR: the slot staged here was last read in iteration kt - 1, whose reads every wave retired
    // (lgkmcnt(0)) before the barrier above
    if (kt + NS - 1 < ksteps) stage_k(kt + NS - 1, slot == 0 ? NS - 1 : slot - 1);
    const char* As = smem + slot * kStage + wm * 64 * 128;
    const char* Bs = smem + slot * kStage + kTileA + wn * 64 * 128;
    slot = slot + 1 == NS ? 0 : slot + 1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = *(const bf16x8*)(As + i * 32 * 128 + aoff[s]);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = *(const bf16x8*)(Bs + j * 32 * 128 + aoff[s]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // Epilogue.  acc[i][j][e]: row m0 + wm*64 + i*32 + (e&3) + 8*(e>>2) + 4*h,
  //                          col n0 + wn*64 + j*32 + r.
  if (PART) {   // raw fp32 partial sums of this split; splitk_epi_kernel finishes
    float* wz = a.ws + (int64_t)blockIdx.z * a.m * a.n;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 64 + j * 32 + r;
      if (col >= a.n) continue;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int64_t row = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (row < a.m) wz[row * a.n + col] = acc[i][j][e];
        }
    }
    return;
  }
  if (m0 + kBM <= a.m && n0 + kBN <= a.n) {
    // full tile: every residual / GELU-input value is loaded before the first store and no element
    // is guarded -- a guarded load per element made hipcc branch around each one and wait for its
    // round trip (64 serial L2 / HBM round trips per thread in the epilogue)
    float aux[2][2][16];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int64_t row = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          const int64_t col = n0 + wn * 64 + j * 32 + r;
          aux[j][i][e] = (EPI & EPI_AUX) ? (float)a.R[row * a.ldr + col] : 0.f;
        }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 64 + j * 32 + r;
      const float bv = (EPI & EPI_BIAS) ? a.bias[col] : 0.0f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int64_t row = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          float v = acc[i][j][e] * a.alpha + bv;
          if (EPI & EPI_PRE) ((__bf16*)a.C2)[row * a.ldc + col] = (__bf16)v;
          if (EPI & EPI_GELU) v = gelu_erf(v);
          v = epi_post<EPI>(a, v, row, col, aux[j][i][e]);
          if (OUT_BF16) ((__bf16*)a.C)[row * a.ldc + col] = (__bf16)v;
          else ((float*)a.C)[row * a.ldc + col] = v;
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t col = n0 + wn * 64 + j * 32 + r;
    if (col >= a.n) continue;
    float bv = 0.0f;
    if (EPI & EPI_BIAS) bv = a.bias[col];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t row = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (row >= a.m) continue;
        float v = acc[i][j][e] * a.alpha + bv;
        if (EPI & EPI_PRE) ((__bf16*)a.C2)[row * a.ldc + col] = (__bf16)v;
        if (EPI & EPI_GELU) v = gelu_erf(v);
        v = epi_post<EPI>(a, v, row, col, (EPI & EPI_AUX) ? (float)a.R[row * a.ldr + col] : 0.f);
        if (OUT_BF16) ((__bf16*)a.C)[row * a.ldc + col] = (__bf16)v;
        else ((float*)a.C)[row * a.ldc + col] = v;
      }
    }
  }
}

// Split-K finish: out = epilogue(sum_z ws[z]) in a fixed z order (deterministic), 4 columns
// per thread when n % 4 == 0.
template <bool OUT_BF16, int EPI>
__global__ __launch_bounds__(256) void splitk_epi_kernel(GemmArgs a, int splits) {
  const int64_t mn = a.m * a.n;
  const bool v4 = (a.n % 4 == 0) && (a.ldc % 4 == 0) && (!(EPI & EPI_AUX) || a.ldr % 4 == 0);
  const int64_t units = v4 ? mn / 4 : mn;
  for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < units; u += (int64_t)gridDim.x * 256) {
    const int64_t e0 = v4 ? u * 4 : u;
    const int64_t row = e0 / a.n, col = e0 % a.n;
    const int w = v4 ? 4 : 1;
    float v[4];
    if (v4) {
      f32x4 s4 = *(const f32x4*)(a.ws + e0);
      for (int z = 1; z < splits; ++z) {
        const f32x4 t = *(const f32x4*)(a.ws + (int64_t)z * mn + e0);
        s4 += t;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = s4[q];
    } else {
      float s1 = a.ws[e0];
      for (int z = 1; z < splits; ++z) s1 += a.ws[(int64_t)z * mn + e0];
      v[0] = s1;
    }
    for (int q = 0; q < w; ++q) {
      float x = v[q] * a.alpha;
      if (EPI & EPI_BIAS) x += a.bias[col + q];
      if (EPI & EPI_PRE) ((__bf16*)a.C2)[row * a.ldc + col + q] = (__bf16)x;
      if (EPI & EPI_GELU) x = gelu_erf(x);
      x = epi_post<EPI>(a, x, row, col + q, (EPI & EPI_AUX) ? (float)a.R[row * a.ldr + col + q] : 0.f);
      if (OUT_BF16) ((__bf16*)a.C)[row * a.ldc + col + q] = (__bf16)x;
      else ((float*)a.C)[row * a.ldc + col + q] = x;
    }
  }
}

// Split-K finish of a pre-LayerNorm sublayer sum fused with that LayerNorm (query-sized batches,
// BertSelfOutput / BertOutput, modeling_bert.py:282-352): per row, x = bf16(sum_z ws[z] * alpha + bias
// + resid) exactly as splitk_epi_kernel<true, EPI_BIAS | EPI_RESID> stores it, then ln_row over those
// values exactly as layernorm_bf16_kernel reads them back: bit-identical to the two launches it
// replaces.  One wave per row (H = 64 * EPL); out may alias resid (a row is read before it is written).
template <int EPL>
__global__ __launch_bounds__(256) void splitk_ln_kernel(const float* ws, int splits, int64_t M, int H, float alpha,
                                                        const float* bias, const __bf16* resid, const float* gamma,
                                                        const float* beta, float eps, __bf16* out) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= M) return;
  const int64_t mn = M * H;
  constexpr int C4 = EPL / 4;
  // the split sums, 4 splits x C4 chunks of loads in flight per step (one wave per row: a serial
  // load-add chain per split would pay one L2 round trip per split and chunk); the additions keep
  // splitk_epi_kernel's z order
  f32x4 s4[C4];
  const float* row = ws + t * H + lane * 4;
#pragma unroll
  for (int e4 = 0; e4 < C4; ++e4) s4[e4] = *(const f32x4*)(row + e4 * 256);
  int z = 1;
  for (; z + 4 <= splits; z += 4) {
    f32x4 q[4][C4];
#pragma unroll
    for (int zz = 0; zz < 4; ++zz)
#pragma unroll
      for (int e4 = 0; e4 < C4; ++e4) q[zz][e4] = *(const f32x4*)(row + (int64_t)(z + zz) * mn + e4 * 256);
#pragma unroll
    for (int zz = 0; zz < 4; ++zz)
#pragma unroll
      for (int e4 = 0; e4 < C4; ++e4) s4[e4] += q[zz][e4];
  }
  for (; z < splits; ++z)
#pragma unroll
    for (int e4 = 0; e4 < C4; ++e4) s4[e4] += *(const f32x4*)(row + (int64_t)z * mn + e4 * 256);
  float x[EPL];
#pragma unroll
  for (int e4 = 0; e4 < C4; ++e4) {
    const int c = e4 * 256 + lane * 4;
    const bf16x4 r = *(const bf16x4*)(resid + t * H + c);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float v = s4[e4][u] * alpha;
      v += bias[c + u];
      v += (float)r[u];
      x[e4 * 4 + u] = (float)(__bf16)v;
    }
  }
  ln_row<EPL>(x, gamma, beta, eps, lane, H, out + t * H);
}

// ---------------------------------------------------------------------------
// GEMM plan: ONE function decides the kernel and the K split of a problem, and both the
// workspace query (drt_linear_workspace) and every launcher use it, so the scratch a caller
// sizes is exactly the scratch the launch writes.
//   LARGE        >= kLargeMinTiles 256^2 tiles: the whole-line 256^2 kernel, unsplit
//   LARGE_SPLIT  long K (>= kLSplitMinK) on a small 256^2 grid: K split so the grid is at most
//                ONE round of blocks (floor(CUs / tiles) splits; a ceiling put e.g. 9 tiles x 29
//                splits = 261 blocks on 256 CUs and the launch took ~2x its one-round time),
//                >= kLSplitKPer per split, fp32 partials <= 256 MiB, fixed-order reduction
//   SMALL_SPLIT  query-sized problems (< 384 tiles of 128^2, K >= 256): 128^2 kernel, splits to
//                about kSmallSplitBlocks blocks, >= 128 K per split, partials <= 16 MiB (at
//                4096 x 768 -- a 128-query batch -- 3 splits = 38 MB of partials measured slower
//                than unsplit)
//   SMALL        everything else (and any split plan whose scratch the caller did not give)
// ---------------------------------------------------------------------------
constexpr int64_t kLSplitMinK = 8192, kLSplitKPer = 512, kSSplitCap = 16 << 20;
// Blocks a SMALL_SPLIT grid aims at.  With the 4-stage ring kernel a block streams its K range
// without waiting on each K-tile, so fewer, longer splits win: query tower at batch 8 (256 tokens)
// 0.827 ms at 512, 0.756 at 32, 0.738 at 64, 0.753 at 96, 0.772 at 128, 0.943 unsplit
// (profiles/r03f_query_encode_*, r03g_query_encode_*); batch 128 unchanged.
constexpr int64_t kSmallSplitBlocks = 64;
enum GemmPath { GP_LARGE, GP_LARGE_SPLIT, GP_SMALL_SPLIT, GP_SMALL };
struct GemmPlan {
  int path = GP_SMALL;
  int splits = 0;
  int64_t kchunk = 0;
  size_t ws_bytes = 0;   // fp32 partials the split needs
};

// Compute units of the current device, looked up once per process.
static int gemm_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, v = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
              ? v
              : 256;
  }
  return cus;
}

// splits -> (splits, kchunk) with kchunk a multiple of `align`; < 2 splits = none
static int round_splits(int64_t k, int64_t splits, int64_t align, int64_t* kchunk) {
  if (splits < 2) return 0;
  int64_t kc = (k + splits - 1) / splits;
  kc = (kc + align - 1) / align * align;
  splits = (k + kc - 1) / kc;
  if (splits < 2) return 0;
  *kchunk = kc;
  return (int)splits;
}

static int large_splits(int64_t m, int64_t n, int64_t k, int64_t* kchunk) {
  const int64_t tiles = ((m + 255) / 256) * ((n + 255) / 256);
  if (tiles >= kLargeMinTiles || k < kLSplitMinK || k % 32) return 0;
  int64_t splits = gemm_cus() / tiles;
  if (splits > k / kLSplitKPer) splits = k / kLSplitKPer;
  const int64_t cap = (int64_t)(256ll << 20) / (m * n * 4);
  if (splits > cap) splits = cap;
  return round_splits(k, splits, 64, kchunk);
}

static int small_splits(int64_t m, int64_t n, int64_t k, int64_t* kchunk) {
  const int64_t tiles = ((m + kBM - 1) / kBM) * ((n + kBN - 1) / kBN);
  if (tiles >= 384 || k < 256) return 0;
  int64_t splits = (kSmallSplitBlocks + tiles - 1) / tiles;
  if (splits > k / 128) splits = k / 128;
  const int64_t cap = kSSplitCap / (m * n * 4);
  if (splits > cap) splits = cap;
  return round_splits(k, splits, kBK, kchunk);
}

static GemmPlan plan_gemm(int64_t m, int64_t n, int64_t k) {
  GemmPlan p;
  if (m <= 0 || n <= 0 || k <= 0) return p;
  const int64_t tiles_l = ((m + kL - 1) / kL) * ((n + kL - 1) / kL);
  if (tiles_l >= kLargeMinTiles) {
    p.path = GP_LARGE;
    return p;
  }
  int64_t kc = 0;
  int s = large_splits(m, n, k, &kc);
  if (s > 1) {
    p.path = GP_LARGE_SPLIT;
  } else {
    s = small_splits(m, n, k, &kc);
    if (s > 1) p.path = GP_SMALL_SPLIT;
  }
  if (s > 1) {
    p.splits = s;
    p.kchunk = kc;
    p.ws_bytes = (size_t)s * (size_t)m * (size_t)n * sizeof(float);
  }
  return p;
}

// The plan a launch actually runs: a split plan degrades to the unsplit 128^2 kernel when the
// caller's scratch is missing or smaller than the plan needs (never writes past ws_bytes).
static GemmPlan plan_for_launch(int64_t m, int64_t n, int64_t k, const void* ws, size_t ws_bytes) {
  GemmPlan p = plan_gemm(m, n, k);
  if (p.splits > 1 && (ws == nullptr || ws_bytes < p.ws_bytes)) p = GemmPlan{};
  return p;
}

// ---------------------------------------------------------------------------
// Ping-pong 256 x 256 kernel (the encoder projections' main path).
//
//  * 8 waves = two groups of 4 (waves 0-3: token rows 0-127 of the tile,
//    waves 4-7: rows 128-255), one wave of each group per SIMD.  Group 1 runs
//    one s_barrier behind group 0, so on every SIMD one wave issues its MFMA
//    cluster while its partner issues the LDS fragment reads and LDS-DMA of the
//    next phase (matrix beside memory, MI355X_MICROARCH.md "Two waves per SIMD").
//  * K is streamed in slabs of 32: one slab = X panel [256 tok][64 B] + W panel
//    [256 out][64 B] = 32 KiB, landed by global_load_lds_dwordx4 into a 4-slot
//    ring (128 KiB), two slabs in flight (counted vmcnt, never 0 in the loop,
//    raw s_barrier).  Each phase issues one panel (2 DMA per wave) of slab s+2.
//  * slab = 2 phases per wave: phase a reads W frags j 0-3 + X frags i 0-3 and
//    issues 16 v_mfma_f32_16x16x32_bf16; phase b reads X frags i 4-7 and issues
//    16 more.  Wave tile = 128 tokens x 64 outputs = 8 x 4 tiles of 16 x 16.
//  * operands swapped (D = W . X^T): lane owns one token row and 4 consecutive
//    output columns per tile -> 8-B bf16 / 16-B fp32 stores.
// Panel image: [row][4 x 16 B], 16-B chunk XOR ((row >> 1) & 2): conflict-free
// ds_read_b128 for the 16x16x32 lane map (row = lane & 15, chunk = lane >> 4).
// WAR/RAW of the ring (group 1 lags one barrier): slab s+2 is waited for in
// phase b of slab s by every wave before the barrier both groups pass before
// reading it; slot (s+2)&3 last held slab s-2, whose final reads retired
// (lgkmcnt(0)) two barriers before the first DMA into it.
// ---------------------------------------------------------------------------
constexpr int kPPanel = kL * 32 * 2;     // 16 KiB
constexpr int kPSlab = 2 * kPPanel;      // 32 KiB
constexpr int kPRing = 4;

// TN operands (weight gradients dW = dY^T X: both stored [t][features], t = the reduction
// index): a 32-t slab of a 256-column panel is 32 rows of 512 B (whole cache lines) in a
// [t][256 cols] image with the 16-B chunk XOR-swizzled by tn_swz(row) = 2 (row & 3) ^ 8 ((row >> 3) & 1);
// the MFMA fragments are read column-wise with ds_read_b64_tr_b16 (two per fragment), which
// this swizzle keeps conflict-free for every 32-lane half.
__device__ __forceinline__ int tn_swz(int row) { return (2 * (row & 3)) ^ (8 * ((row >> 3) & 1)); }

// 32 t-rows x 256 columns into the swizzled [t][512 B] image: 16 wave-instructions of 2 rows, 2 per wave.
// Columns past `cols` are clamped to the last whole chunk (their outputs are masked).
__device__ __forceinline__ void stage_panel32_tn(const __bf16* base, int64_t ld, int64_t col0, int64_t cols,
                                                 int64_t t0, uint32_t lds, int wave, int lane) {
  const int cp = lane & 31;   // chunk position in the LDS row
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int J = j * 8 + wave;
    const int row = 2 * J + (lane >> 5);
    int64_t col = col0 + (int64_t)((cp ^ tn_swz(row)) * 8);
    col = col + 8 <= cols ? col : cols - 8;
    g_glds16(base + (t0 + row) * ld + col, __builtin_amdgcn_readfirstlane(lds + J * 1024));
  }
}

typedef short tn_v4i16 __attribute__((ext_vector_type(4)));

// 16x16x32 operand fragment of columns [cb, cb + 16) (cb % 16 == 0, cb < 256) from a TN image:
// lane l gets column cb + (l & 15), t rows 8 (l >> 4) .. +7.  rowoff = byte offset of row
// 8 (l >> 4) + ((l & 15) >> 2) (the second read is 4 rows below), s = tn_swz of that row,
// lo = 16 ((l & 3) >> 1) + 8 (l & 1).
__device__ __forceinline__ bf16x8 tn_frag(const char* img, int cb, int rowoff, int s, int lo) {
  const int off = rowoff + ((((cb >> 3)) ^ s) << 4) + lo;
  typedef __attribute__((address_space(3))) tn_v4i16 lds_v4;
  const tn_v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(uintptr_t)g_lds_addr(img + off));
  const tn_v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(uintptr_t)g_lds_addr(img + off + 4 * 512));
  bf16x8 r;
  __builtin_memcpy(&r, &a, 8);
  __builtin_memcpy((char*)&r + 8, &b, 8);
  return r;
}

// Tile order inside the contiguous range of tiles an XCD owns (wg = rank in the
// XCD-remapped grid): 0 row-major (consecutive tiles share the X panel),
// 1 grouped by 8 m-panels (a round of 32 concurrent tiles = 8 m x 4 n panels),
// 2 column-major inside the XCD's m-range (a round shares one W panel),
// 3 / 4 grouped by 4 / 16 m-panels.
__device__ __forceinline__ void tile_order(int order, int wg, int nwg, int tiles_n, int& tm, int& tn) {
  if (order == 0) {
    tm = wg / tiles_n;
    tn = wg % tiles_n;
    return;
  }
  const int tiles_m = nwg / tiles_n;
  if (order == 1 || order >= 3) {
    const int G = order == 1 ? 8 : (order == 3 ? 4 : 16);
    const int grp = wg / (G * tiles_n), first = grp * G;
    const int gm = tiles_m - first < G ? tiles_m - first : G;
    const int l = wg - grp * G * tiles_n;
    tm = first + l % gm;
    tn = l / gm;
    return;
  }
  // order 2: the XCD's m-range is [x*mpx, ...); walk it column by column
  const int mpx = (tiles_m + 7) / 8;
  const int x = wg / (mpx * tiles_n);
  const int first = x * mpx;
  const int gm = tiles_m - first < mpx ? tiles_m - first : mpx;
  const int l = wg - x * mpx * tiles_n;
  tm = first + l % gm;
  tn = l / gm;
}

// s_waitcnt vmcnt(4 * n): all but the n youngest slabs (4 LDS-DMA per wave each) landed.
__device__ __forceinline__ void vmcnt_slabs_after(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
  }
}

template <bool OUT_BF16, int EPI>
__device__ __forceinline__ void pp_epilogue(const GemmArgs& a, f32x4 (&acc)[8][4], int64_t m0, int64_t n0, int grp,
                                            int wn, int fr, int fc) {
  // Epilogue. acc[i][j][u]: token row m0 + grp*128 + i*16 + fr,
  //                         output col n0 + wn*64 + j*16 + 4*fc + u.
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t col = n0 + wn * 64 + j * 16 + 4 * fc;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t row = m0 + grp * 128 + i * 16 + fr;
      if (row >= a.m) continue;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (col + u >= a.n) continue;
        float x = acc[i][j][u] * a.alpha + ((EPI & EPI_BIAS) ? a.bias[col + u] : 0.f);
        if (EPI & EPI_PRE) ((__bf16*)a.C2)[row * a.ldc + col + u] = (__bf16)x;
        if (EPI & EPI_GELU) x = gelu_erf(x);
        x = epi_post<EPI>(a, x, row, col + u, (EPI & EPI_AUX) ? (float)a.R[row * a.ldr + col + u] : 0.f);
        if (OUT_BF16) ((__bf16*)a.C)[row * a.ldc + col + u] = (__bf16)x;
        else ((float*)a.C)[row * a.ldc + col + u] = x;
      }
    }
  }
}

// Epilogue through LDS (T21-style widening): each wave stages its 128 x 64 output
// slice in a private LDS region (row-per-lane 8-B pieces in, 16-B row-contiguous
// pieces out, 16-B chunks XOR-swizzled by row), then writes whole 128-B (bf16) /
// 256-B (fp32) row segments.  Needs a full tile in n; rows are masked.
// bf16 outputs leave as non-temporal stores (round 6): every CU's 128 KiB tile per round is an
// XCD's whole 4 MB L2, and plain stores evicted the X / W panels the next round's tiles re-read
// (encode 38.6-39.0k -> 39.6-39.8k passages/s in three alternating rounds, FFN2 -8 %, FFN1 -3 %,
// outputs bit-identical; profiles/r06v/).
template <bool OUT_BF16, int EPI>
__device__ __forceinline__ void pp_epilogue_lds(const GemmArgs& a, f32x4 (&acc)[8][4], int64_t m0, int64_t n0,
                                                int grp, int wn, int fr, int fc, char* lds_wave, int lane) {
  const int64_t colw = n0 + wn * 64;   // first column of this wave's slice
  f32x4 bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (EPI & EPI_BIAS) bv[j] = *(const f32x4*)(a.bias + colw + j * 16 + 4 * fc);
  }
  if (OUT_BF16 && !(EPI & (EPI_AUX | EPI_DROP))) {
    // [128 rows][8 x 16 B], chunk ^= row & 7; EPI_PRE: a first pass stores the pre-activation
#pragma unroll
    for (int pass = (EPI & EPI_PRE) ? 0 : 1; pass < 2; ++pass) {
      const bool act = pass == 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = i * 16 + fr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bf16x4 o;
#pragma unroll
          for (int u = 0; u < 4; u += 2) {   // element pairs: the GELU on packed fp32 math
            f32x2 x = {acc[i][j][u] * a.alpha + bv[j][u], acc[i][j][u + 1] * a.alpha + bv[j][u + 1]};
            if ((EPI & EPI_GELU) && act) x = gelu_fast2(x);
            o[u] = (__bf16)x.x;
            o[u + 1] = (__bf16)x.y;
          }
          const int chunk = (2 * j + (fc >> 1)) ^ (r & 7);
          *(bf16x4*)(lds_wave + r * 128 + chunk * 16 + (fc & 1) * 8) = o;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      const int c = lane & 7;
      __bf16* dst = act ? (__bf16*)a.C : (__bf16*)a.C2;
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        const int r = p * 8 + (lane >> 3);
        const bf16x8 v = *(const bf16x8*)(lds_wave + r * 128 + ((c ^ (r & 7)) << 4));
        const int64_t row = m0 + grp * 128 + r;
        if (row < a.m) __builtin_nontemporal_store(v, (bf16x8*)(dst + row * a.ldc + colw + c * 8));
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
  } else {
    // two passes of 64 rows: [64 rows][16 x 16 B] fp32, chunk ^= row & 7, read back as 8
    // consecutive columns per lane (two chunks: conflict-free for every ds_read_b128 lane group),
    // so residual loads and bf16 stores are 16 B per lane (fp32 stores 2 x 16 B).  bf16 output
    // with a residual (pre-LayerNorm sums) stages fp32, so the sum is rounded once, at the store.
    // Residual rows of pass 1 are requested once pass 0 is staged (its accumulators are dead).
    const int c8 = lane & 7;
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // csum: this lane's 8 columns
    bf16x8 rq[2][8];
    auto load_rq = [&](int h) {
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        int64_t row = m0 + grp * 128 + h * 64 + p * 8 + (lane >> 3);
        row = row < a.m ? row : a.m - 1;
        rq[h][p] = *(const bf16x8*)(a.R + row * a.ldr + colw + c8 * 8);
      }
    };
    if (EPI & EPI_AUX) load_rq(0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = i * 16 + fr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4 v;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            float x = acc[h * 4 + i][j][u] * a.alpha + bv[j][u];
            if ((EPI & EPI_PRE) && m0 + grp * 128 + h * 64 + r < a.m)
              ((__bf16*)a.C2)[(m0 + grp * 128 + h * 64 + r) * a.ldc + colw + j * 16 + 4 * fc + u] = (__bf16)x;
            if (EPI & EPI_GELU) x = gelu_fast(x);
            v[u] = x;
          }
          const int chunk = (j * 4 + fc) ^ (r & 7);
          *(f32x4*)(lds_wave + r * 256 + chunk * 16) = v;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      if ((EPI & EPI_AUX) && h == 0) load_rq(1);
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const int r = p * 8 + (lane >> 3);
        const f32x4 v0 = *(const f32x4*)(lds_wave + r * 256 + (((2 * c8) ^ (r & 7)) << 4));
        const f32x4 v1 = *(const f32x4*)(lds_wave + r * 256 + (((2 * c8 + 1) ^ (r & 7)) << 4));
        const int64_t row = m0 + grp * 128 + h * 64 + r;
        if (row < a.m) {
          float v[8];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            v[u] = v0[u];
            v[4 + u] = v1[u];
          }
          if (EPI & (EPI_AUX | EPI_DROP)) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
              v[u] = epi_post<EPI>(a, v[u], row, colw + c8 * 8 + u, (EPI & EPI_AUX) ? (float)rq[h][p][u] : 0.f);
          }
          if (OUT_BF16) {
            bf16x8 o;
#pragma unroll
            for (int u = 0; u < 8; ++u) o[u] = (__bf16)v[u];
            __builtin_nontemporal_store(o, (bf16x8*)((__bf16*)a.C + row * a.ldc + colw + c8 * 8));
            if (a.csum) {
#pragma unroll
              for (int u = 0; u < 8; ++u) cs[u] += (float)o[u];
            }
          } else {
            *(f32x4*)((float*)a.C + row * a.ldc + colw + c8 * 8) = f32x4{v[0], v[1], v[2], v[3]};
            *(f32x4*)((float*)a.C + row * a.ldc + colw + c8 * 8 + 4) = f32x4{v[4], v[5], v[6], v[7]};
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
    if (OUT_BF16 && a.csum) {   // the 8 lanes of each column group hold 16 rows each: xor 8 / 16 / 32
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float x = cs[u];
        x += __shfl_xor(x, 8, 64);
        x += __shfl_xor(x, 16, 64);
        x += __shfl_xor(x, 32, 64);
        cs[u] = x;
      }
      if (lane < 8) {
        float* dst = a.csum + ((m0 / 256) * 2 + grp) * a.n + colw + c8 * 8;
        *(f32x4*)dst = f32x4{cs[0], cs[1], cs[2], cs[3]};
        *(f32x4*)(dst + 4) = f32x4{cs[4], cs[5], cs[6], cs[7]};
      }
    }
  }
}

// Weight-gradient (TN) kernel: dW = dY^T X with both operands token-major.  One phase per
// 32-token slab: per wave, a memory segment (12 column-wise fragment reads of slab s,
// LDS-DMA of slab s+4, vmcnt for slab s+1, lgkmcnt(0)) and a 32-MFMA segment, ping-ponged
// with the partner wave of the other group.  Because the reading wave drains its own
// fragment reads before the barrier that ends its memory segment, the ring slot of slab s
// is free one barrier later: 5 slots carry 4 slabs in flight (128 KiB per CU).
// RAW: slab s+1 is waited for (vmcnt) in the memory segment of slab s by every wave, before
// the barrier after which group 0 reads it.  WAR: slot (s+4) % 5 held slab s-1, whose reads
// both groups drained before the barrier that precedes group 0's memory segment of slab s.
constexpr int kTnRing = 5;
__global__ __launch_bounds__(kLThreads, 1) void gemm_tn_kernel(GemmArgs a) {
  constexpr int RING = kTnRing, D = RING - 1;   // slabs in flight
  __shared__ __attribute__((aligned(16))) char smem[RING * kPSlab];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int grp = wave >> 2;
  const int wn = wave & 3;

  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tiles_n = (int)((a.n + kL - 1) / kL);
  int tm, tn;
  tile_order(a.order, wg, nwg, tiles_n, tm, tn);
  const int64_t m0 = (int64_t)tm * kL;
  const int64_t n0 = (int64_t)tn * kL;

  const uint32_t lds0 = g_lds_addr(smem);
  // split over tokens (kchunk > 0): this block sums t in [kb, kb + kchunk) of split blockIdx.y and
  // stores raw fp32 partials at C + blockIdx.y * m * ldc (splitk_epi_kernel finishes)
  const int64_t kb = a.kchunk ? (int64_t)blockIdx.y * a.kchunk : 0;
  const int64_t ke = a.kchunk ? (kb + a.kchunk < a.k ? kb + a.kchunk : a.k) : a.k;
  const int ns = (int)((ke - kb) / 32);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fc = lane >> 4;
  // fragment addressing (tn_frag): row 8 fc + (fr >> 2), chunk half (fr & 3) >> 1, 8-B half fr & 1
  const int tn_row = 8 * fc + (fr >> 2);
  const int tn_rowoff = tn_row * 512, tn_s = tn_swz(tn_row), tn_lo = 16 * ((fr & 3) >> 1) + 8 * (fr & 1);
  auto stage = [&](int64_t t0, uint32_t dst) {
    stage_panel32_tn(a.A, a.lda, m0, a.m, t0, dst, wave, lane);
    stage_panel32_tn(a.B, a.ldb, n0, a.n, t0, dst + kPPanel, wave, lane);
  };

  // prologue: slabs 0..D-1 in flight, slab 0 landed
#pragma unroll
  for (int p = 0; p < D; ++p) {
    if (p < ns) stage(kb + p * 32, lds0 + p * kPSlab);
  }
  vmcnt_slabs_after(ns - 1 < D - 1 ? ns - 1 : D - 1);
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  int slot = 0, fill = D % RING;
  for (int s = 0; s < ns; ++s) {
    const char* slab = smem + slot * kPSlab;
    // ---- memory segment
    bf16x8 wf[4], xf[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[j] = tn_frag(slab + kPPanel, wn * 64 + j * 16, tn_rowoff, tn_s, tn_lo);
#pragma unroll
    for (int i = 0; i < 8; ++i) xf[i] = tn_frag(slab, grp * 128 + i * 16, tn_rowoff, tn_s, tn_lo);
    const int left = ns - 1 - s;   // slabs after s
    if (left >= D) {
      stage(kb + (int64_t)(s + D) * 32, lds0 + fill * kPSlab);
      vmcnt_slabs_after(D - 1);
    } else {
      vmcnt_slabs_after(left > 0 ? left - 1 : 0);
    }
    slot = slot + 1 == RING ? 0 : slot + 1;
    fill = fill + 1 == RING ? 0 : fill + 1;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---- matrix segment
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();
  GemmArgs ae = a;
  if (a.kchunk) ae.C = (float*)a.C + (int64_t)blockIdx.y * a.m * a.ldc;
  const bool full = (n0 + kL <= a.n) && (a.ldc % 8 == 0);
  if (full) pp_epilogue_lds<false, EPI_NONE>(ae, acc, m0, n0, grp, wn, fr, fc, smem + wave * 16384, lane);
  else pp_epilogue<false, EPI_NONE>(ae, acc, m0, n0, grp, wn, fr, fc);
}

// ---------------------------------------------------------------------------
// Whole-line K-tiles (the encoder projections' main path since round 2).
//
// pp1 lands 32-deep slabs: every LDS-DMA wave-instruction covers 16 rows x 64 B, i.e. 16
// HALF cache lines (the fragment-shaped pattern that doubles TA work per byte).  Here a
// K-tile is 64 deep: one wave-instruction = 8 rows x 128 B (whole lines), panel image
// [256 rows][8 x 16 B] with the 16-B chunk XOR (row & 7) (conflict-free ds_read_b128 for
// every lane group of the 16x16x32 fragment map).  Measured on the way (tools/gemm_ab.py,
// profiles/r02m_gemm_ab.log): the same ping-pong on two 64-KiB K-tile buffers (8 DMA per
// wave in one memory segment, none in the other) gained only 1-6 % over pp1; the panel ring
// below spreads them 4 + 4 and gains 5-18 %; a persistent form of the ring (panel stream
// across tiles, next tile's first panels landing during the epilogue) measured no faster.
// ---------------------------------------------------------------------------
constexpr int kQPanel = kL * 128;        // 32 KiB: 256 rows x 64 k

// 256 rows x 64 k into a [row][8 x 16 B] panel (chunk ^= row & 7): 32 wave-instructions
// of 8 whole rows, 4 per wave.  Lane l covers row 8J + (l >> 3), chunk (l & 7) ^ (l >> 3): its
// byte offset from the wave-uniform row-block address is a per-lane constant (one VGPR), the
// block address lives in SGPRs.  Rows past `rows` are clamped (masked in the epilogue): only a
// row block that crosses `rows` takes the per-lane clamp.
__device__ __forceinline__ int panel64_lane_off(int64_t ld, int lane) {
  const int rsub = lane >> 3;
  return (int)(rsub * ld * 2) + (((lane & 7) ^ rsub) << 4);
}
__device__ __forceinline__ void stage_panel64(const __bf16* base, int64_t ld, int64_t row0, int64_t rows,
                                              int64_t k0, uint32_t lds, int wave, int lane, int lane_off) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int J = j * 8 + wave;           // 0..31
    const int64_t r = row0 + J * 8;       // wave-uniform
    const char* p = (const char*)(base + r * ld + k0);
    int off = lane_off;
    if (r + 8 > rows) {
      const int rsub = lane >> 3;
      const int64_t gr = r + rsub < rows ? r + rsub : rows - 1;
      off = (int)((gr - r) * ld * 2) + (((lane & 7) ^ rsub) << 4);
    }
    g_glds16(p + off, __builtin_amdgcn_readfirstlane(lds + J * 1024));
  }
}

// ---------------------------------------------------------------------------
// Whole-line K-tiles in a 5-slot PANEL ring (160 KiB): the unit of the ring is one
// operand panel of one K-tile (X_t or W_t, [256 rows][128 B] = 32 KiB), panel P = 2t + op
// in slot P mod 5.  While tile t is read (its 2 panels), the other 3 slots take W_{t+1}
// and X_{t+2}: X panels land 1.5 K-tiles ahead, W panels one ahead, and every memory
// segment carries 4 LDS-DMA per wave (the 2-buffer form carried 8, then 0).
//   mem(t,0): 12 fragment reads (k-half 0) + W_{t+1} (into X_{t-1}'s slot)
//   mat(t,0): 32 MFMA
//   mem(t,1): 12 fragment reads (k-half 1) + X_{t+2} (into W_{t-1}'s slot), then
//             vmcnt(4): X_{t+1} and W_{t+1} landed (X_{t+2} may stay in flight)
//   mat(t,1): 32 MFMA
// G1 one barrier behind G0 as in pp1.  WAR: X_{t-1} and W_{t-1} were last read in
// G1's mem(t-1,1) (interval 4t-1), drained before the barrier that opens 4t, the first
// interval in which any wave stages into their slots.  RAW: both groups wait in their
// mem(t,1) (intervals 4t+2 / 4t+3) before the barrier that closes 4t+3; tile t+1 is first
// read in 4t+4.
// ---------------------------------------------------------------------------
template <bool OUT_BF16, int EPI>
__global__ __launch_bounds__(kLThreads, 1) void gemm_nt_pr5_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[5 * kQPanel];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int grp = wave >> 2;
  const int wn = wave & 3;

  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tiles_n = (int)((a.n + kL - 1) / kL);
  int tm, tn;
  tile_order(a.order, wg, nwg, tiles_n, tm, tn);
  const int64_t m0 = (int64_t)tm * kL;
  const int64_t n0 = (int64_t)tn * kL;
  const uint32_t lds0 = g_lds_addr(smem);
  // split-K (kchunk > 0): this block sums k in [kb, kb + kchunk) of split blockIdx.y and stores raw
  // fp32 partials at C + blockIdx.y * m * ldc (splitk_epi_kernel finishes in a fixed split order)
  const int64_t kb = a.kchunk ? (int64_t)blockIdx.y * a.kchunk : 0;
  const int64_t ke = a.kchunk ? (kb + a.kchunk < a.k ? kb + a.kchunk : a.k) : a.k;
  const int nt = (int)((ke - kb) / 64);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fc = lane >> 4;
  const int foff0 = fr * 128 + ((fc ^ (fr & 7)) << 4);
  const int foff1 = fr * 128 + (((4 + fc) ^ (fr & 7)) << 4);
  const int loffA = panel64_lane_off(a.lda, lane), loffB = panel64_lane_off(a.ldb, lane);
  const int xrow = grp * 128 * 128;
  const int wrow = wn * 64 * 128;
  auto stage_x = [&](int t, int slot) {
    stage_panel64(a.A, a.lda, m0, a.m, kb + (int64_t)t * 64, lds0 + slot * kQPanel, wave, lane, loffA);
  };
  auto stage_w = [&](int t, int slot) {
    stage_panel64(a.B, a.ldb, n0, a.n, kb + (int64_t)t * 64, lds0 + slot * kQPanel, wave, lane, loffB);
  };

  // prologue: X_0 (slot 0), W_0 (slot 1) landed, X_1 (slot 2) in flight
  stage_x(0, 0);
  stage_w(0, 1);
  if (nt > 1) {
    stage_x(1, 2);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  int xs = 0;   // slot of X_t = 2t mod 5; W_t in xs + 1 (mod 5)
  for (int t = 0; t < nt; ++t) {
    const int ws = xs == 4 ? 0 : xs + 1;
    const char* X = smem + xs * kQPanel + xrow;
    const char* W = smem + ws * kQPanel + wrow;
    bf16x8 wf[4], xf[8];
    // ---- phase 0: memory segment (+ W_{t+1} into slot 2t+3 mod 5)
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[j] = *(const bf16x8*)(W + j * 16 * 128 + foff0);
#pragma unroll
    for (int i = 0; i < 8; ++i) xf[i] = *(const bf16x8*)(X + i * 16 * 128 + foff0);
    if (t + 1 < nt) stage_w(t + 1, xs + 3 >= 5 ? xs - 2 : xs + 3);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 1: memory segment (+ X_{t+2} into slot 2t+4 mod 5, then wait for tile t+1)
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[j] = *(const bf16x8*)(W + j * 16 * 128 + foff1);
#pragma unroll
    for (int i = 0; i < 8; ++i) xf[i] = *(const bf16x8*)(X + i * 16 * 128 + foff1);
    if (t + 2 < nt) {
      stage_x(t + 2, xs + 4 >= 5 ? xs - 1 : xs + 4);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    xs = xs + 2 >= 5 ? xs - 3 : xs + 2;
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();
  GemmArgs ae = a;
  if (a.kchunk) ae.C = (float*)a.C + (int64_t)blockIdx.y * a.m * a.ldc;
  const bool full = (n0 + kL <= a.n) && (a.ldc % 8 == 0) && (!(EPI & EPI_AUX) || a.ldr % 8 == 0);
  if (full) pp_epilogue_lds<OUT_BF16, EPI>(ae, acc, m0, n0, grp, wn, fr, fc, smem + wave * 16384, lane);
  else pp_epilogue<OUT_BF16, EPI>(ae, acc, m0, n0, grp, wn, fr, fc);
}

static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Finish a split: out = epilogue(sum_z ws[z]) in a fixed z order.
template <bool OUT_BF16, int EPI>
static void launch_splitk_epi(const GemmArgs& a, int splits, hipStream_t s) {
  const int64_t units = (a.n % 4 == 0) ? a.m * a.n / 4 : a.m * a.n;
  const int64_t blocks = ceil_div(units, 256) < 4096 ? ceil_div(units, 256) : 4096;
  hipLaunchKernelGGL((splitk_epi_kernel<OUT_BF16, EPI>), dim3((unsigned)blocks), dim3(256), 0, s, a, splits);
}

// The 128^2 kernel: the 4-stage ring when the grid fits in one round of CUs (one block per CU),
// the double buffer otherwise.  Same K order and MFMA sequence: bit-identical outputs.
template <bool OUT_BF16, int EPI, bool PART>
static void launch_small(const GemmArgs& a, int64_t tiles, int splits, hipStream_t s) {
  const dim3 grid((unsigned)tiles, 1, (unsigned)splits);
  if (tiles * splits <= gemm_cus())
    hipLaunchKernelGGL((gemm_nt_kernel<OUT_BF16, EPI, PART, 4>), grid, dim3(kGemmThreads), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<OUT_BF16, EPI, PART, 2>), grid, dim3(kGemmThreads), 0, s, a);
}

template <bool OUT_BF16, int EPI>
static int launch_gemm_t(const GemmArgs& a0, size_t ws_bytes, hipStream_t s) {
  GemmArgs a = a0;
  a.order = auto_tile_order(a.k);
  const GemmPlan p = plan_for_launch(a.m, a.n, a.k, a.ws, ws_bytes);
  const ProfPair pp = prof_begin(PROF_GEMM, s);
  const int64_t tiles_l = ceil_div(a.m, kL) * ceil_div(a.n, kL);
  const int64_t tiles = ceil_div(a.m, kBM) * ceil_div(a.n, kBN);
  switch (p.path) {
    case GP_LARGE:
      // whole-line K-tiles in the 5-slot panel ring (tools/gemm_ab.py: +5-18 % over the 32-deep
      // slab ring, bit-identical outputs)
      hipLaunchKernelGGL((gemm_nt_pr5_kernel<OUT_BF16, EPI>), dim3((unsigned)tiles_l), dim3(kLThreads), 0, s, a);
      break;
    case GP_LARGE_SPLIT: {
      // long K, small output: raw fp32 partials per split, then one fixed-order reduction
      // applying the epilogue
      GemmArgs b = a;
      b.kchunk = p.kchunk;
      b.C = a.ws;
      b.ldc = a.n;
      b.bias = nullptr;
      b.R = nullptr;
      b.alpha = 1.0f;
      hipLaunchKernelGGL((gemm_nt_pr5_kernel<false, EPI_NONE>), dim3((unsigned)tiles_l, (unsigned)p.splits),
                         dim3(kLThreads), 0, s, b);
      launch_splitk_epi<OUT_BF16, EPI>(a, p.splits, s);
      break;
    }
    case GP_SMALL_SPLIT: {
      GemmArgs b = a;
      b.kchunk = p.kchunk;
      launch_small<OUT_BF16, EPI, true>(b, tiles, p.splits, s);
      launch_splitk_epi<OUT_BF16, EPI>(b, p.splits, s);
      break;
    }
    default:
      launch_small<OUT_BF16, EPI, false>(a, tiles, 1, s);
      break;
  }
  prof_end(pp, s);
  return hip_status(hipGetLastError());
}

int launch_gemm(const GemmArgs& a, bool out_bf16, int epi, size_t ws_bytes, hipStream_t s) {
  if (a.m == 0 || a.n == 0) return DRT_OK;
  if (a.k <= 0 || a.k % kBK != 0) return DRT_EINVAL;
  if (!out_bf16) {
    switch (epi) {
      case EPI_NONE: return launch_gemm_t<false, EPI_NONE>(a, ws_bytes, s);
      case EPI_BIAS: return launch_gemm_t<false, EPI_BIAS>(a, ws_bytes, s);
      case EPI_BIAS | EPI_RESID: return launch_gemm_t<false, EPI_BIAS | EPI_RESID>(a, ws_bytes, s);
      case EPI_RESID: return launch_gemm_t<false, EPI_RESID>(a, ws_bytes, s);
      default: return DRT_EINVAL;
    }
  }
  switch (epi) {
    case EPI_NONE: return launch_gemm_t<true, EPI_NONE>(a, ws_bytes, s);
    case EPI_BIAS: return launch_gemm_t<true, EPI_BIAS>(a, ws_bytes, s);
    case EPI_BIAS | EPI_GELU: return launch_gemm_t<true, EPI_BIAS | EPI_GELU>(a, ws_bytes, s);
    case EPI_BIAS | EPI_RESID: return launch_gemm_t<true, EPI_BIAS | EPI_RESID>(a, ws_bytes, s);
    case EPI_RESID: return launch_gemm_t<true, EPI_RESID>(a, ws_bytes, s);   // backward dgrad + residual branch
    case EPI_GELU: return launch_gemm_t<true, EPI_GELU>(a, ws_bytes, s);
    // training tower fusions (drt_linear_bf16_ex)
    case EPI_BIAS | EPI_GELU | EPI_PRE: return launch_gemm_t<true, EPI_BIAS | EPI_GELU | EPI_PRE>(a, ws_bytes, s);
    case EPI_DGELU: return launch_gemm_t<true, EPI_DGELU>(a, ws_bytes, s);
    case EPI_BIAS | EPI_DROP | EPI_RESID: return launch_gemm_t<true, EPI_BIAS | EPI_DROP | EPI_RESID>(a, ws_bytes, s);
    default: return DRT_EINVAL;
  }
}

}  // namespace drt

using namespace drt;

extern "C" int drt_gemm_nt_bf16_f32(const void* A, const void* B, float* C, int64_t m, int64_t n, int32_t d,
                                    int64_t ldc, void* stream) {
  DRT_REQUIRE(m >= 0 && n >= 0 && d > 0 && d % 64 == 0 && ldc >= n);
  if (m == 0 || n == 0) return DRT_OK;
  DRT_REQUIRE(A && B && C);
  GemmArgs a{};
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = C;
  a.m = m;
  a.n = n;
  a.k = d;
  a.lda = d;
  a.ldb = d;
  a.ldc = ldc;
  a.alpha = 1.0f;
  return launch_gemm(a, false, EPI_NONE, 0, (hipStream_t)stream);
}

// Workspace that lets drt_linear_bf16_ws / _ln_ / _ex split K on problems too small to fill the
// chip: exactly the plan's fp32 partials (0 when the plan does not split this shape).
extern "C" size_t drt_linear_workspace(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64) return 0;
  return plan_gemm(M, N, K).ws_bytes;
}

extern "C" int drt_linear_bf16_ws(const void* X, const void* W, const float* bias, const void* residual, void* Y,
                                  int64_t M, int64_t N, int64_t K, int32_t flags, void* ws, size_t ws_bytes,
                                  void* stream);

// nn.Linear: Y[M, N] = X[M, K] . W[N, K]^T (+ bias) (GELU) (+ residual [M, N] bf16)
// flags: DRT_LIN_GELU = 1, DRT_LIN_OUT_F32 = 2.
extern "C" int drt_linear_bf16(const void* X, const void* W, const float* bias, const void* residual, void* Y,
                               int64_t M, int64_t N, int64_t K, int32_t flags, void* stream) {
  return drt_linear_bf16_ws(X, W, bias, residual, Y, M, N, K, flags, nullptr, 0, stream);
}

extern "C" int drt_linear_bf16_ws(const void* X, const void* W, const float* bias, const void* residual, void* Y,
                                  int64_t M, int64_t N, int64_t K, int32_t flags, void* ws, size_t ws_bytes,
                                  void* stream) {
  DRT_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 64 == 0);
  if (M == 0) return DRT_OK;
  DRT_REQUIRE(X && W && Y);
  const bool gelu = flags & 1, f32 = flags & 2;
  DRT_REQUIRE(!(gelu && residual));
  GemmArgs a{};
  a.A = (const __bf16*)X;
  a.B = (const __bf16*)W;
  a.C = Y;
  a.bias = bias;
  a.R = (const __bf16*)residual;
  a.m = M;
  a.n = N;
  a.k = K;
  a.lda = K;
  a.ldb = K;
  a.ldc = N;
  a.ldr = N;
  a.alpha = 1.0f;
  a.ws = (float*)ws;
  const int epi = (bias ? EPI_BIAS : 0) | (gelu ? EPI_GELU : 0) | (residual ? EPI_RESID : 0);
  return launch_gemm(a, !f32, epi, ws ? ws_bytes : 0, (hipStream_t)stream);
}

extern "C" int drt_layernorm_bf16(const void* X, int64_t M, int32_t H, const float* gamma, const float* beta, float eps,
                                  void* out, void* stream);

// LayerNorm(bf16(X W^T + bias + residual)) -> out (BertSelfOutput / BertOutput: dense + residual +
// LayerNorm).  When the plan is the 128^2 split (query-sized batches, caller scratch >=
// drt_linear_workspace) the K-split partials are finished by one fused split-K + LayerNorm launch
// (splitk_ln_kernel); otherwise the linear writes its bf16 pre-LayerNorm sum to `presum` and
// drt_layernorm_bf16 normalises it.  Either way bit-identical to drt_linear_bf16_ws + drt_layernorm_bf16.
// out may alias residual.  N % 256 == 0, N <= 1024.
extern "C" int drt_linear_ln_bf16_ws(const void* X, const void* W, const float* bias, const void* residual,
                                     const float* gamma, const float* beta, float eps, void* presum, void* out,
                                     int64_t M, int64_t N, int64_t K, void* ws, size_t ws_bytes, void* stream) {
  DRT_REQUIRE(M >= 0 && N > 0 && N % 256 == 0 && N <= 1024 && K > 0 && K % 64 == 0);
  if (M == 0) return DRT_OK;
  DRT_REQUIRE(X && W && bias && residual && gamma && beta && presum && out);
  hipStream_t s = (hipStream_t)stream;
  const GemmPlan p = plan_for_launch(M, N, K, ws, ws ? ws_bytes : 0);
  if (p.path != GP_SMALL_SPLIT) {
    const int rc = drt_linear_bf16_ws(X, W, bias, residual, presum, M, N, K, 0, ws, ws_bytes, stream);
    if (rc != DRT_OK) return rc;
    return drt_layernorm_bf16(presum, M, (int32_t)N, gamma, beta, eps, out, stream);
  }
  GemmArgs b{};
  b.A = (const __bf16*)X;
  b.B = (const __bf16*)W;
  b.C = presum;   // unused by the partial kernel (PART writes b.ws)
  b.m = M;
  b.n = N;
  b.k = K;
  b.lda = K;
  b.ldb = K;
  b.ldc = N;
  b.ldr = N;
  b.alpha = 1.0f;
  b.ws = (float*)ws;
  b.kchunk = p.kchunk;
  b.order = auto_tile_order(K);
  const int64_t tiles = ceil_div(M, kBM) * ceil_div(N, kBN);
  const ProfPair pp = prof_begin(PROF_GEMM, s);
  launch_small<true, EPI_BIAS | EPI_RESID, true>(b, tiles, p.splits, s);
  const dim3 grid((unsigned)((M + 3) / 4));
  const int splits = p.splits;
  switch (N / 64) {
    case 4: hipLaunchKernelGGL(splitk_ln_kernel<4>, grid, dim3(256), 0, s, (const float*)ws, splits, M, (int)N, 1.0f,
                               bias, (const __bf16*)residual, gamma, beta, eps, (__bf16*)out); break;
    case 8: hipLaunchKernelGGL(splitk_ln_kernel<8>, grid, dim3(256), 0, s, (const float*)ws, splits, M, (int)N, 1.0f,
                               bias, (const __bf16*)residual, gamma, beta, eps, (__bf16*)out); break;
    case 12: hipLaunchKernelGGL(splitk_ln_kernel<12>, grid, dim3(256), 0, s, (const float*)ws, splits, M, (int)N, 1.0f,
                                bias, (const __bf16*)residual, gamma, beta, eps, (__bf16*)out); break;
    case 16: hipLaunchKernelGGL(splitk_ln_kernel<16>, grid, dim3(256), 0, s, (const float*)ws, splits, M, (int)N, 1.0f,
                                bias, (const __bf16*)residual, gamma, beta, eps, (__bf16*)out); break;
    default: return DRT_EINVAL;
  }
  prof_end(pp, s);
  return hip_status(hipGetLastError());
}

// drt_linear_bf16_ws plus the training tower's epilogue fusions (include/drt.h):
//   gelu_pre != NULL: Y = (X W^T) * GELU'(gelu_pre)  (the dgrad through GELU; no bias / residual / GELU);
//   Y_pre != NULL (with GELU): Y_pre = X W^T + b, Y = GELU(Y_pre)  (both bf16);
//   flags & 4 (DROP): Y = dropout(X W^T + b) + residual with drt_dropout_add_bf16's mask of (seed, site).
// The split plan is the same as drt_linear_bf16_ws's (plan_gemm), so drt_linear_workspace sizes it.
extern "C" int drt_linear_bf16_ex(const void* X, const void* W, const float* bias, const void* residual,
                                  const void* gelu_pre, void* Y, void* Y_pre, int64_t M, int64_t N, int64_t K,
                                  int32_t flags, float drop_p, uint64_t seed, uint64_t site, void* ws,
                                  size_t ws_bytes, void* stream) {
  DRT_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 64 == 0);
  if (M == 0) return DRT_OK;
  DRT_REQUIRE(X && W && Y);
  const bool gelu = flags & 1, f32 = flags & 2, drop = flags & 4;
  DRT_REQUIRE(!f32 || (!gelu_pre && !Y_pre && !drop));
  DRT_REQUIRE(!gelu_pre || (!bias && !residual && !gelu && !Y_pre && !drop));
  DRT_REQUIRE(!Y_pre || (gelu && !residual && !drop));
  DRT_REQUIRE(!drop || (drop_p >= 0.f && drop_p < 1.f && !gelu));
  GemmArgs a{};
  a.A = (const __bf16*)X;
  a.B = (const __bf16*)W;
  a.C = Y;
  a.C2 = Y_pre;
  a.bias = bias;
  a.R = (const __bf16*)(gelu_pre ? gelu_pre : residual);
  a.m = M;
  a.n = N;
  a.k = K;
  a.lda = K;
  a.ldb = K;
  a.ldc = N;
  a.ldr = N;
  a.alpha = 1.0f;
  a.drop_p = drop_p;
  a.seed = seed;
  a.site = site;
  a.ws = (float*)ws;
  const int epi = (bias ? EPI_BIAS : 0) | (gelu ? EPI_GELU : 0) | (residual ? EPI_RESID : 0) |
                  (gelu_pre ? EPI_DGELU : 0) | (Y_pre ? EPI_PRE : 0) | (drop ? EPI_DROP : 0);
  return launch_gemm(a, !f32, epi, ws ? ws_bytes : 0, (hipStream_t)stream);
}

// FFN1 dgrad with the GELU backward AND its bias gradient: dX = (dY W^T) * GELU'(pre) (bf16, as
// drt_linear_bf16_ex with gelu_pre), dbias[N] = column sums of the stored dX.  On the whole-line
// plan with full column tiles the GEMM epilogue leaves per-half-tile column sums (no pass over dX);
// otherwise dX is summed after the GEMM.  ws: the GEMM's split partials, then the column-sum
// partials and their reduction scratch.
static bool dgelu_fused(int64_t M, int64_t N, int64_t K) {
  return plan_gemm(M, N, K).path == GP_LARGE && N % kL == 0;
}
extern "C" size_t drt_linear_dgelu_bias_workspace(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64) return 0;
  const size_t g = (plan_gemm(M, N, K).ws_bytes + 255) & ~(size_t)255;
  if (dgelu_fused(M, N, K)) {
    const int64_t rows = 2 * ceil_div(M, kL);
    return g + (size_t)rows * N * sizeof(float) + drt_colsum_workspace(rows, N);
  }
  return g + drt_colsum_workspace(M, N);
}

extern "C" int drt_linear_dgelu_bias_bf16(const void* dY, const void* Wt, const void* gelu_pre, void* dX, int64_t M,
                                          int64_t N, int64_t K, float* dbias, void* ws, size_t ws_bytes,
                                          void* stream) {
  DRT_REQUIRE(M > 0 && N > 0 && K > 0 && K % 64 == 0 && dY && Wt && gelu_pre && dX && dbias);
  DRT_REQUIRE(ws_bytes >= drt_linear_dgelu_bias_workspace(M, N, K) && (ws || ws_bytes == 0));
  hipStream_t s = (hipStream_t)stream;
  const size_t g = (plan_gemm(M, N, K).ws_bytes + 255) & ~(size_t)255;
  char* rest = (char*)ws + g;
  GemmArgs a{};
  a.A = (const __bf16*)dY;
  a.B = (const __bf16*)Wt;
  a.C = dX;
  a.R = (const __bf16*)gelu_pre;
  a.m = M;
  a.n = N;
  a.k = K;
  a.lda = K;
  a.ldb = K;
  a.ldc = N;
  a.ldr = N;
  a.alpha = 1.0f;
  a.ws = (float*)ws;
  if (dgelu_fused(M, N, K)) {
    const int64_t rows = 2 * ceil_div(M, kL);
    a.csum = (float*)rest;
    int rc = launch_gemm(a, true, EPI_DGELU, g, s);
    if (rc) return rc;
    return drt_colsum_f32(a.csum, rows, N, dbias, rest + (size_t)rows * N * sizeof(float),
                          drt_colsum_workspace(rows, N), stream);
  }
  int rc = launch_gemm(a, true, EPI_DGELU, g, s);
  if (rc) return rc;
  return drt_colsum_bf16(dX, M, N, dbias, rest, drt_colsum_workspace(M, N), stream);
}

// Weight gradient of nn.Linear without transposed operand copies: dW[N][K] fp32 = dY[T][N]^T . X[T][K]
// (both operands stored token-major, as the backward has them).  The 256^2 ping-pong TN kernel
// (whole-line slabs, ds_read_b64_tr_b16 fragments), K = T split over ~1 block per CU with fp32
// partials in ws reduced in a fixed order (deterministic): the LARGE_SPLIT plan of plan_gemm.
extern "C" size_t drt_linear_wgrad_workspace(int64_t T, int64_t N, int64_t K) {
  if (T <= 0 || N <= 0 || K <= 0 || T % 32 || N % 8 || K % 8) return 0;
  int64_t kc = 0;
  const int ls = large_splits(N, K, T, &kc);
  return ls > 1 ? (size_t)ls * (size_t)N * (size_t)K * sizeof(float) : 0;
}

extern "C" int drt_linear_wgrad_bf16(const void* dY, const void* X, float* dW, int64_t T, int64_t N, int64_t K,
                                     void* ws, size_t ws_bytes, void* stream) {
  DRT_REQUIRE(T > 0 && N >= 8 && K >= 8 && T % 32 == 0 && N % 8 == 0 && K % 8 == 0);
  DRT_REQUIRE(dY && X && dW);
  hipStream_t s = (hipStream_t)stream;
  GemmArgs a{};
  a.A = (const __bf16*)dY;
  a.B = (const __bf16*)X;
  a.C = dW;
  a.m = N;
  a.n = K;
  a.k = T;
  a.lda = N;
  a.ldb = K;
  a.ldc = K;
  a.alpha = 1.0f;
  a.order = auto_tile_order(T);
  const int64_t tiles_l = ceil_div(N, kL) * ceil_div(K, kL);
  int64_t kc = 0;
  const int splits = large_splits(N, K, T, &kc);
  if (splits > 1) DRT_REQUIRE(ws && ws_bytes >= (size_t)splits * (size_t)N * (size_t)K * sizeof(float));
  const ProfPair pp = prof_begin(PROF_GEMM, s);
  if (splits > 1) {
    GemmArgs b = a;
    b.kchunk = kc;
    b.C = ws;
    hipLaunchKernelGGL(gemm_tn_kernel, dim3((unsigned)tiles_l, (unsigned)splits), dim3(kLThreads), 0, s, b);
    GemmArgs e = a;
    e.ws = (float*)ws;
    launch_splitk_epi<false, EPI_NONE>(e, splits, s);
  } else {
    hipLaunchKernelGGL(gemm_tn_kernel, dim3((unsigned)tiles_l), dim3(kLThreads), 0, s, a);
  }
  prof_end(pp, s);
  return hip_status(hipGetLastError());
}
