// Backward building blocks of the bi-encoder tower (the training step of
// run_random_sampling.py, DRT/trainer/trainer.py:113-133 -> DRModel.forward -> HF BertModel
// under autograd).  Each kernel restates the gradient of one forward op of
// transformers modeling_bert.py (BertSelfOutput / BertOutput LayerNorm :282-352,
// BertIntermediate GELU :325-337, nn.Linear bias) for the bf16 activations the HIP forward
// stores; the tower-level assembly (with dropout masks) is the next step.
//
//   layernorm_bwd   dx = rstd (g - mean(g) - xhat mean(g xhat)),  g = dy * gamma,
//                   (+ a residual gradient), per-block dgamma / dbeta partials
//   colsum          out[n] = sum_rows x[row][n] in a fixed order (bias / LN parameter grads)
//   gelu_bwd        dx = dy (Phi(x) + x phi(x))      (erf GELU, activations.py:70-90)
//   transpose_bf16  y[c][r] = x[r][c]                 (operand layout for weight gradients)
//   attention_bwd   dQ, dK, dV of softmax(Q K^T / sqrt(dh) + mask) V  (L <= 160)
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
// partial sums in part[blockIdx.x][0..H) and part[gridDim.x + blockIdx.x][0..H); SUM: also the
// column sums of the gradient handed down (dxd when dropping, else dx, as stored in bf16) in
// part[2 gridDim.x + blockIdx.x] -- the bias gradient of the linear below, without a pass
// that reads that gradient again.
template <int EPL, bool SUM>
__global__ __launch_bounds__(256, EPL <= 12 ? 4 : 1) void layernorm_bwd_kernel(const __bf16* dy, const __bf16* x, const float* gamma,
                                                            float eps, int64_t M, int H, const __bf16* dres,
                                                            __bf16* dx, float* part, __bf16* dxd, float drop_p,
                                                            uint64_t seed, uint64_t site) {
  __shared__ float red[4][SUM ? 3 : 2][EPL * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // SUM keeps 4 wave-wide partial sums per column: gamma is re-read per row there (an L1 hit)
  // instead of held in registers, so the kernel keeps 4 waves per SIMD without spilling
  float dg[EPL], db[EPL], gm[SUM ? 1 : EPL], ds[SUM ? EPL : 1];
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    dg[e] = 0.f;
    db[e] = 0.f;
    if (SUM) ds[SUM ? e : 0] = 0.f;
    else gm[SUM ? 0 : e] = gamma[(e >> 2) * 256 + lane * 4 + (e & 3)];
  }
  for (int64_t t = (int64_t)blockIdx.x * 4 + wave; t < M; t += (int64_t)gridDim.x * 4) {
    float xv[EPL], gv[EPL], dyv[EPL], gmr[SUM ? EPL : 1];
#pragma unroll
    for (int e4 = 0; e4 < EPL / 4; ++e4) {
      const int c = e4 * 256 + lane * 4;
      const bf16x4 a = *(const bf16x4*)(x + t * H + c);
      const bf16x4 b = *(const bf16x4*)(dy + t * H + c);
      f32x4 g4 = {};
      if (SUM) g4 = *(const f32x4*)(gamma + c);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        xv[e4 * 4 + u] = (float)a[u];
        dyv[e4 * 4 + u] = (float)b[u];
        if (SUM) gmr[SUM ? e4 * 4 + u : 0] = g4[u];
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
      gv[e] = dyv[e] * (SUM ? gmr[SUM ? e : 0] : gm[SUM ? 0 : e]);
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
      if (dxd) {   // dropout of the rounded dx (what drt_dropout_add_bf16 would compute from it)
        const uint32_t thr = drop_threshold(drop_p);
        const float inv = 1.0f / (1.0f - drop_p);
        bf16x4 od;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool keep = drop_hash24(seed, site, (uint64_t)(t * H + c + u)) >= thr;
          od[u] = (__bf16)(keep ? (float)o[u] * inv : 0.0f);
          if (SUM) ds[SUM ? e4 * 4 + u : 0] += (float)od[u];
        }
        *(bf16x4*)(dxd + t * H + c) = od;
      } else if (SUM) {
#pragma unroll
        for (int u = 0; u < 4; ++u) ds[SUM ? e4 * 4 + u : 0] += (float)o[u];
      }
    }
  }
  // fixed-order block reduction of the 4 waves' parameter-gradient sums
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    red[wave][0][e * 64 + lane] = dg[e];
    red[wave][1][e * 64 + lane] = db[e];
    if (SUM) red[wave][SUM ? 2 : 0][e * 64 + lane] = ds[SUM ? e : 0];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < EPL * 64; i += 256) {
    const int e = i >> 6, ln = i & 63;
    const int col = (e >> 2) * 256 + ln * 4 + (e & 3);
    part[(int64_t)blockIdx.x * H + col] = ((red[0][0][i] + red[1][0][i]) + red[2][0][i]) + red[3][0][i];
    part[(int64_t)(gridDim.x + blockIdx.x) * H + col] = ((red[0][1][i] + red[1][1][i]) + red[2][1][i]) + red[3][1][i];
    if (SUM) {
      constexpr int k = SUM ? 2 : 0;
      part[(int64_t)(2 * gridDim.x + blockIdx.x) * H + col] = ((red[0][k][i] + red[1][k][i]) + red[2][k][i]) + red[3][k][i];
    }
  }
}

// out[n] = sum over rows [0, M) of x[row][n]: stage 1 (this kernel with FINAL = false) sums
// row slabs into part[slab][n]; stage 2 (FINAL = true) sums the slabs in order.  fp32 sums.
// out[y][n] = sum of x[row][n] over the rows [y * rows_per, (y + 1) * rows_per) of slab y.
// A wave covers 64 x VEC consecutive columns with 16-B loads (1 KiB per row per instruction);
// the block's 4 waves take every 4th row of the slab and are added in a fixed order at the end
// (deterministic).  Columns: full 16-B vectors when N % VEC == 0, element-wise otherwise.
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* x, int64_t M, int64_t N, int64_t rows_per,
                                                     float* out) {
  constexpr int VEC = 16 / (int)sizeof(T);
  __shared__ float red[3][64 * VEC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c0 = ((int64_t)blockIdx.x * 64 + lane) * VEC;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = r0 + rows_per < M ? r0 + rows_per : M;
  float acc[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
  if (c0 < N) {
    if (N % VEC == 0) {
      typedef T tv __attribute__((ext_vector_type(VEC)));
      int64_t r = r0 + wave;
#pragma unroll 4
      for (; r < r1; r += 4) {
        const tv val = *(const tv*)(x + r * N + c0);
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v] += (float)val[v];
      }
    } else {
      for (int64_t r = r0 + wave; r < r1; r += 4)
#pragma unroll
        for (int v = 0; v < VEC; ++v)
          if (c0 + v < N) acc[v] += (float)x[r * N + c0 + v];
    }
  }
  if (wave > 0) {
#pragma unroll
    for (int v = 0; v < VEC; ++v) red[wave - 1][lane * VEC + v] = acc[v];
  }
  __syncthreads();
  if (wave == 0 && c0 < N) {
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const float t = ((acc[v] + red[0][lane * VEC + v]) + red[1][lane * VEC + v]) + red[2][lane * VEC + v];
      if (c0 + v < N) out[(int64_t)blockIdx.y * N + c0 + v] = t;
    }
  }
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

// 64 x 64 tiles through LDS.  Full tiles (R, C multiples of 8): 16-B global loads of input
// rows and 16-B stores of output rows (8 lanes per 128-B output segment), LDS rows padded to
// 144 B (16-B aligned); edge tiles take the element-wise path.  y has row stride ldy >= R.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const __bf16* x, int64_t R, int64_t C, __bf16* y,
                                                             int64_t ldy) {
  __shared__ __attribute__((aligned(16))) __bf16 t[64][72];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tid = threadIdx.x;
  const bool full = r0 + 64 <= R && c0 + 64 <= C && (C & 7) == 0 && (ldy & 7) == 0;
  if (full) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int idx = tid + it * 256, row = idx >> 3, ch = idx & 7;
      *(bf16x8*)&t[row][ch * 8] = *(const bf16x8*)(x + (r0 + row) * C + c0 + ch * 8);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int idx = tid + it * 256, j = idx & 7, c = idx >> 3;   // output row c0 + c, rows r0 + 8j..+7
      bf16x8 v;
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = t[8 * j + u][c];
      *(bf16x8*)(y + (c0 + c) * ldy + r0 + 8 * j) = v;
    }
    return;
  }
  const int tx = tid & 63, ty = tid >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    t[i][tx] = (r < R && c < C) ? x[r * C + c] : (__bf16)0.0f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < C && r < R) y[c * ldy + r] = t[tx][i];
  }
}

// ---------------------------------------------------------------------------
// Attention backward (BertSelfAttention, modeling_bert.py:164-204, under autograd), one
// work-group per (sequence, head), L <= 160 (the reference recipe's p_max_len 156, run.sh),
// head_dim 64.  With Qs = scale * Q (rounded to bf16 as the forward does), S = Qs K^T + key bias,
// P = exp(S - lse):
//   Dv_q = sum_d dO[q][d] O[q][d];   dP = dO V^T;   dS = P (dP - Dv)
//   dV = P^T dO;   dK = dS^T Qs;   dQ = scale * dS K.
// With dropout, O = Pd V where Pd = mask P / (1 - p): dV takes Pd, and dS = P (mask dP / (1 - p) - Dv).
// LDS: Qs, K, V, dO row-major [Lp][64] (16-B chunk XOR (row >> 1) & 7, as the forward's K image),
// read row-wise with ds_read_b128 (operands along d) and column-wise with ds_read_b64_tr_b16 (the
// B operands of dV, dK, dQ along the sequence: no transposed copies).  Each phase computes its
// score tile in the orientation whose MFMA output layout IS the A operand of the next product,
// so P / dS never go through LDS:
//   phase 1 (wave = key block kbk, loop over query blocks):  S = Qs K^T and dP = dO V^T as
//     [query rows (registers)][key (lane)] tiles; a lane then holds, for its key, 16 queries of the
//     block -- exactly the A operand of dV = Pd^T dO and dK = dS^T Qs with the k (query) order
//     permuted (8 (e >> 2) + 4 h + (e & 3)); the B operands are read in the same permuted row order
//     with ds_read_b64_tr_b16 (rows base + 4 h .. + 3 and base + 8 + 4 h .. + 3).
//   phase 2 (wave = query block, loop over key blocks): S^T = K Qs^T and dP^T = V dO^T as
//     [key rows][query (lane)] tiles = the A operand of dQ = dS K (k = key, permuted likewise).
// The key-block operands of phase 1 (K, V as B operands) and the query-block operands of phase 2
// (Qs, dO) stay in registers for the whole phase.  Per-query values of phase 1 (lse, Dv, keep words)
// are read as 16-B vectors, four queries at a time.  DROP: the forward's keep bits (drop_bits)
// staged in LDS as [key block][query] words; C-ABI callers without them get the same words drawn
// again from the pairwise hash (drt_common.h attn_row_key / attn_mix) while staging.
// 32x32x16 MFMA: A lane (m = l & 31, h = l >> 5) holds A[m][k = 8h .. 8h + 7]; B lane (n, h) holds
// B[k = 8h ..][n]; D lane (n = l & 31, h) holds D[m = 8 (e >> 2) + 4 h + (e & 3)][n].
// ---------------------------------------------------------------------------
constexpr int kAbMaxSeq = 160;
constexpr int kAbRow = 128;               // bytes per [.][64] bf16 row


struct AttnBwdArgs {
  const __bf16* qkv;     // [B*L][3H]
  const __bf16* ctx;     // [B*L][H]  forward output O
  const __bf16* dctx;    // [B*L][H]  dO
  const float* lse;      // [B][heads][L]
  const int64_t* mask;   // [B][L] or null
  __bf16* dqkv;          // [B*L][3H]
  int64_t B, L;
  int heads, H;
  float scale;
  float drop_p;           // attention-probability dropout of the forward (0: none)
  uint64_t seed, site;
  const uint32_t* drop_bits;  // optional keep bits written by the forward ([B][heads][L][ceil(L/32)]);
                              // NULL: the same bits drawn again from the hash
  float* dsum;                // optional [B][3H] (L > 160: [B][ceil(L / 128)][3H]): column sums of dQKV
};

__device__ __forceinline__ int ab_rc(int row, int chunk) { return row * kAbRow + ((chunk ^ ((row >> 1) & 7)) << 4); }

typedef short ab_v4i16 __attribute__((ext_vector_type(4)));

// Per-lane LDS offsets of the fragment reads, fixed for the kernel: every row block starts at a
// multiple of 32 rows, so the swizzle term (row >> 1) & 7 of a block's row never depends on the
// block (16 blk = 0 mod 8).  A-operand rows (blk * 32 + r, chunk 2 k4 + h): offA[k4]; column-wise
// B operands (ab_tr8p rows blk * 32 + 16 ks + 4 h + q and + 8, col0 = 32 t): offT[t][0 / 1].
// A read of block blk is then img + blk * 4096 (+ ks * 2048) + offset: with NB a template
// argument and the block loops unrolled, one VGPR + an immediate per read.
struct AbOffsets {
  int offA[4];
  int offT[2][2];
};
__device__ __forceinline__ AbOffsets ab_offsets(int lane) {
  AbOffsets o;
  const int r = lane & 31, h = lane >> 5, sw = (r >> 1) & 7;
#pragma unroll
  for (int k4 = 0; k4 < 4; ++k4) o.offA[k4] = r * kAbRow + (((2 * k4 + h) ^ sw) << 4);
  const int i = lane & 15, q = i >> 2, p = i & 3, b4 = (lane >> 4) & 1;
  const int sx = 2 * h + (q >> 1), lo = (p & 1) * 8;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int c = 4 * t + 2 * b4 + (p >> 1);
    o.offT[t][0] = (q + 4 * h) * kAbRow + ((c ^ sx) << 4) + lo;
    o.offT[t][1] = (q + 4 * h + 8) * kAbRow + ((c ^ (sx + 4)) << 4) + lo;
  }
  return o;
}

__device__ __forceinline__ bf16x8 ab_tr8o(const char* img, int off0, int off1) {
  typedef __attribute__((address_space(3))) ab_v4i16 lds_v4;
  const ab_v4i16 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(img + off0));
  const ab_v4i16 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(img + off1));
  bf16x8 v;
  __builtin_memcpy(&v, &x, 8);
  __builtin_memcpy((char*)&v + 8, &y, 8);
  return v;
}

// Per-score-element work of the two phases on element PAIRS (v_pk_fma_f32 / v_pk_add_f32 /
// v_pk_mul_f32 issue two fp32 lanes each; exp2 stays per element):
//   P1 (lane = key, 4 queries e0..e0+3): P = exp2(S log2e + (kbias - lse2)), dS = P (keep dP / (1-p) - Dv)
//   P2 (lane = query, 4 keys e0..e0+3):  P = exp2(S log2e + (kb2 - lse2)),   dS = P (keep dP / (1-p) - Dv)
// Same roundings as the per-element form: fma(S, log2e, kbias - lse2) vs fma(S, log2e, kbias) - lse2 can
// differ in the last bit of the exponent argument (checked against torch fp32, not bitwise).
template <bool DROP>
__device__ __forceinline__ void ab_p1_pairs(const f32x16& sv, const f32x16& dp, int e0, const f32x4& lq,
                                            const f32x4& dq, float kbias, const u32x4& wk, uint32_t lanebit,
                                            float inv, bf16x8 (&pa)[2], bf16x8 (&sa)[2]) {
  const f32x2 l2e = {kLog2e, kLog2e}, kb = {kbias, kbias}, iv = {inv, inv};
#pragma unroll
  for (int u = 0; u < 4; u += 2) {
    const int e = e0 + u;
    const f32x2 c = kb - f32x2{lq[u], lq[u + 1]};
    f32x2 x = __builtin_elementwise_fma(f32x2{sv[e], sv[e + 1]}, l2e, c);
    f32x2 p = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
    f32x2 ds, pd = p;
    const f32x2 nd = -f32x2{dq[u], dq[u + 1]};
    if (DROP) {
      const bool k0 = (wk[u] & lanebit) != 0u, k1 = (wk[u + 1] & lanebit) != 0u;
      pd = f32x2{k0 ? p[0] : 0.f, k1 ? p[1] : 0.f};
      ds = p * __builtin_elementwise_fma(f32x2{k0 ? dp[e] : 0.f, k1 ? dp[e + 1] : 0.f}, iv, nd);
    } else {
      ds = p * (f32x2{dp[e], dp[e + 1]} + nd);
    }
    pa[e >> 3][e & 7] = (__bf16)pd[0];
    pa[e >> 3][(e & 7) + 1] = (__bf16)pd[1];
    sa[e >> 3][e & 7] = (__bf16)ds[0];
    sa[e >> 3][(e & 7) + 1] = (__bf16)ds[1];
  }
}

// wbits: bit u (u < 4) = keep of key e0 + u's pair element for this lane's query
template <bool DROP>
__device__ __forceinline__ void ab_p2_pairs(const f32x16& st, const f32x16& dpt, int e0, const f32x4& kbv, float lq,
                                            float dq, uint32_t wbits, float inv, bf16x8 (&sa)[2]) {
  const f32x2 l2e = {kLog2e, kLog2e}, lq2 = {lq, lq}, nd = {-dq, -dq}, iv = {inv, inv};
#pragma unroll
  for (int u = 0; u < 4; u += 2) {
    const int e = e0 + u;
    const f32x2 c = f32x2{kbv[u], kbv[u + 1]} - lq2;
    const f32x2 x = __builtin_elementwise_fma(f32x2{st[e], st[e + 1]}, l2e, c);
    const f32x2 p = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
    f32x2 ds;
    if (DROP) {
      const f32x2 kd = {(wbits >> u) & 1u ? dpt[e] : 0.f, (wbits >> (u + 1)) & 1u ? dpt[e + 1] : 0.f};
      ds = p * __builtin_elementwise_fma(kd, iv, nd);
    } else {
      ds = p * (f32x2{dpt[e], dpt[e + 1]} + nd);
    }
    sa[e >> 3][e & 7] = (__bf16)ds[0];
    sa[e >> 3][(e & 7) + 1] = (__bf16)ds[1];
  }
}

// NB = row blocks of 32 (Lp = 32 NB), NW = waves: one work-group per (sequence, head).
// Exponentials as exp2(s log2e + kb2 - lse2) with the key bias and lse pre-scaled by log2e in
// staging (one fma + one sub + v_exp per score); the dropout scale 1 / (1 - p) leaves the
// per-element path: dS = P (keep ? dP : 0) / (1 - p) - P Dv is one fma on the kept dP, and
// dV = (1 / (1 - p)) sum_q (keep P)^T dO scales the accumulator once at the store.
template <int NB, bool DROP>
__global__ __launch_bounds__((NB == 5 ? 8 : 4) * 64, NB == 5 ? 1 : 2) void attention_bwd_rk_kernel(AttnBwdArgs a) {
  constexpr int NW = NB == 5 ? 8 : 4;
  constexpr int NT = NW * 64;
  constexpr int Lp = NB * 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int L = (int)a.L;
  char* Qs = smem;                                   // [Lp][64] (scaled Q)
  char* Ks = Qs + Lp * kAbRow;
  char* Vs = Ks + Lp * kAbRow;
  char* Os = Vs + Lp * kAbRow;                       // dO
  float* lse2 = (float*)(Os + Lp * kAbRow);          // [Lp]  lse * log2e
  float* dv = lse2 + Lp;                             // [Lp]  Dv
  float* kb2 = dv + Lp;                              // [Lp]  key bias (0 / -FLT_MAX)
  uint32_t* kbits = (uint32_t*)(kb2 + Lp);           // [NB][Lp] keep words (DROP)

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t b = blockIdx.x / a.heads;
  const int hd = blockIdx.x % a.heads;
  const int64_t row0 = b * a.L;
  const int64_t ld = 3 * (int64_t)a.H;
  const __bf16* Qg = a.qkv + row0 * ld + hd * 64;
  const __bf16* Kg = Qg + a.H;
  const __bf16* Vg = Qg + 2 * a.H;
  const __bf16* Og = a.ctx + row0 * a.H + hd * 64;
  const __bf16* dOg = a.dctx + row0 * a.H + hd * 64;

  // ---- staging: every global load of the work-group (the rows of Q, K, V, dO, O, and the per-row
  // lse, mask and keep words) in flight before the first LDS store -- one latency round, which is
  // exposed whenever one work-group holds the CU (L > 128)
  {
    constexpr int MAXIT = (Lp * 8 + NT - 1) / NT;
    constexpr int MAXS = (Lp + NT - 1) / NT;                        // per-row values per thread
    constexpr int MAXW = DROP ? (NB * Lp + NT - 1) / NT : 1;        // keep words
    const int64_t hrow = ((int64_t)b * a.heads + hd) * a.L;
    bf16x8 q[MAXIT], k[MAXIT], v[MAXIT], o[MAXIT], oo[MAXIT];
    float lsev[MAXS];
    int64_t mk[MAXS];
    uint32_t wd[MAXW];
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      const int i = tid + it * NT;
      const int row = i >> 3, c = i & 7;
      q[it] = bf16x8{};
      k[it] = bf16x8{};
      v[it] = bf16x8{};
      o[it] = bf16x8{};
      oo[it] = bf16x8{};
      if (i < Lp * 8 && row < L) {
        q[it] = *(const bf16x8*)(Qg + (int64_t)row * ld + c * 8);
        k[it] = *(const bf16x8*)(Kg + (int64_t)row * ld + c * 8);
        v[it] = *(const bf16x8*)(Vg + (int64_t)row * ld + c * 8);
        o[it] = *(const bf16x8*)(dOg + (int64_t)row * a.H + c * 8);
        oo[it] = *(const bf16x8*)(Og + (int64_t)row * a.H + c * 8);
      }
    }
#pragma unroll
    for (int j = 0; j < MAXS; ++j) {
      const int i = tid + j * NT;
      lsev[j] = 0.0f;
      mk[j] = 1;
      if (i < L) {
        lsev[j] = a.lse[hrow + i];
        if (a.mask) mk[j] = a.mask[b * a.L + i];
      }
    }
    // [query][key block] words of the forward, read in their own order (coalesced)
    const uint32_t* src = DROP && a.drop_bits ? a.drop_bits + hrow * NB : nullptr;
#pragma unroll
    for (int j = 0; j < MAXW; ++j) {
      const int i = tid + j * NT;
      wd[j] = 0u;
      if (src && i < L * NB) wd[j] = src[i];
    }
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      const int i = tid + it * NT;
      if (i >= Lp * 8) break;
      const int row = i >> 3, c = i & 7;
      float part = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        q[it][j] = (__bf16)((float)q[it][j] * a.scale);
        part += (float)o[it][j] * (float)oo[it][j];
      }
      *(bf16x8*)(Qs + ab_rc(row, c)) = q[it];
      *(bf16x8*)(Ks + ab_rc(row, c)) = k[it];
      *(bf16x8*)(Vs + ab_rc(row, c)) = v[it];
      *(bf16x8*)(Os + ab_rc(row, c)) = o[it];
      part += __shfl_xor(part, 1, 64);
      part += __shfl_xor(part, 2, 64);
      part += __shfl_xor(part, 4, 64);
      if (c == 0) dv[row] = part;
    }
#pragma unroll
    for (int j = 0; j < MAXS; ++j) {
      const int i = tid + j * NT;
      if (i < Lp) {
        kb2[i] = (i >= L || mk[j] == 0) ? -3.402823466e+38f : 0.0f;   // (1 - mask) * finfo.min (finite)
        lse2[i] = lsev[j] * kLog2e;
      }
    }
    if (DROP) {   // -> [key block][query]; without the forward's words (drop_bits NULL) the same
                  // words are drawn again from the pairwise hash
      const uint32_t thr = attn_drop_threshold(a.drop_p);
#pragma unroll
      for (int j = 0; j < MAXW; ++j) {
        const int i = tid + j * NT;
        if (i >= NB * Lp) break;
        const int qq = i / NB, kbi = i - qq * NB;
        uint32_t w = wd[j];
        if (!src && qq < L) {
          const uint32_t rk = attn_row_key(a.seed, a.site, (uint64_t)(hrow + qq));
          for (int jj = 0; jj < 16; ++jj) {
            const uint32_t hsh = attn_mix(rk + (uint32_t)(kbi * 16 + jj) * kAttnPairStep);
            const int key = kbi * 32 + 2 * jj;
            w |= (key < L && (hsh & 0xFFFFu) >= thr) ? 1u << (2 * jj) : 0u;
            w |= (key + 1 < L && (hsh >> 16) >= thr) ? 2u << (2 * jj) : 0u;
          }
        }
        kbits[kbi * Lp + qq] = qq < L ? w : 0u;
      }
    }
  }
  __syncthreads();

  const float inv = DROP ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const AbOffsets off = ab_offsets(lane);
  const uint32_t lanebit = 1u << r;

  // Work units: P1(k) = dK, dV of key block k (loop over the query blocks), P2(q) = dQ of query
  // block q (loop over the key blocks).  After staging the LDS images are read-only, so the two
  // kinds run concurrently, each wave through its own list:
  //   NB <= 4 (4 waves): wave w runs P1(w) then P2(w) -- every SIMD the same load;
  //   NB = 5 (8 waves; wave w on SIMD w % 4): w0 P1(0) | w1 P1(1) P2(3) | w2 P1(2) P2(4) |
  //     w3 P1(3) | w4 P1(4) | w5 P2(0) | w6 P2(1) | w7 P2(2): SIMD loads (16 MFMA per P1 step,
  //     12 per P2 step) 32 / 40 / 40 / 28 against 56 on SIMD 0 for phase 1 on waves 0-4 followed
  //     by phase 2 on waves 0-4.
  // Outputs stay in registers (bf16) until every unit is done, then leave through LDS (dK into
  // the Qs image, dV into the dO image, dQ into the K image) as whole 128-B rows of 16-B stores
  // (12 per thread at L 128 instead of 96 two-byte stores per wave).
  int p1 = -1, p2 = -1;
  if (NB <= 4) {
    if (wave < NB) p1 = p2 = wave;
  } else {
    p1 = wave < 5 ? wave : -1;
    p2 = wave >= 5 ? wave - 5 : (wave == 1 ? 3 : (wave == 2 ? 4 : -1));
  }
  bf16x8 dKo[2][2], dVo[2][2], dQo[2][2];             // [t][e >> 3]: element e of column 32 t + r

  // ---- P1: dK, dV of key block p1
  if (p1 >= 0) {
    const int blk = p1;
    const int key = blk * 32 + r;                     // this lane's key (D column / A row)
    bf16x8 kf[4], vf[4];                              // B operands of S = Qs K^T, dP = dO V^T
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
      kf[k4] = *(const bf16x8*)(Ks + blk * 4096 + off.offA[k4]);
      vf[k4] = *(const bf16x8*)(Vs + blk * 4096 + off.offA[k4]);
    }
    const float kbias = kb2[key];
    f32x16 dK[2], dV[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        dK[t][e] = 0.f;
        dV[t][e] = 0.f;
      }
#pragma unroll
    for (int qb = 0; qb < NB; ++qb) {
      f32x16 sv, dp;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        sv[e] = 0.f;
        dp[e] = 0.f;
      }
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const bf16x8 qa = *(const bf16x8*)(Qs + qb * 4096 + off.offA[k4]);
        sv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[k4], sv, 0, 0, 0);
        const bf16x8 oa = *(const bf16x8*)(Os + qb * 4096 + off.offA[k4]);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(oa, vf[k4], dp, 0, 0, 0);
      }
      // P, dS for this lane's key and its 16 queries (four groups of four consecutive queries)
      bf16x8 pa[2], sa[2];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int q0 = qb * 32 + 8 * g + 4 * h;
        const f32x4 lq = *(const f32x4*)(lse2 + q0);
        const f32x4 dq = *(const f32x4*)(dv + q0);
        u32x4 wk = {};
        if (DROP) wk = *(const u32x4*)(kbits + blk * Lp + q0);
        ab_p1_pairs<DROP>(sv, dp, 4 * g, lq, dq, kbias, wk, lanebit, inv, pa, sa);
      }
      // dV += Pd^T dO, dK += dS^T Qs over the block's 32 queries (2 k-steps of 16, permuted rows)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int base = qb * 4096 + ks * 2048;
          const bf16x8 ob = ab_tr8o(Os + base, off.offT[t][0], off.offT[t][1]);
          dV[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa[ks], ob, dV[t], 0, 0, 0);
          const bf16x8 qb8 = ab_tr8o(Qs + base, off.offT[t][0], off.offT[t][1]);
          dK[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sa[ks], qb8, dK[t], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        dKo[t][e >> 3][e & 7] = (__bf16)dK[t][e];
        dVo[t][e >> 3][e & 7] = (__bf16)(DROP ? dV[t][e] * inv : dV[t][e]);
      }
  }

  // ---- P2: dQ of query block p2
  if (p2 >= 0) {
    const int blk = p2;
    const int q = blk * 32 + r;                        // this lane's query (D column)
    bf16x8 qf[4], of[4];                               // B operands of S^T = K Qs^T, dP^T = V dO^T
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
      qf[k4] = *(const bf16x8*)(Qs + blk * 4096 + off.offA[k4]);
      of[k4] = *(const bf16x8*)(Os + blk * 4096 + off.offA[k4]);
    }
    const float lq = lse2[q], dq = dv[q];
    f32x16 dQ[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) dQ[t][e] = 0.f;
#pragma unroll
    for (int kbk = 0; kbk < NB; ++kbk) {
      f32x16 st, dpt;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        st[e] = 0.f;
        dpt[e] = 0.f;
      }
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const bf16x8 ka = *(const bf16x8*)(Ks + kbk * 4096 + off.offA[k4]);
        st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[k4], st, 0, 0, 0);
        const bf16x8 va = *(const bf16x8*)(Vs + kbk * 4096 + off.offA[k4]);
        dpt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, of[k4], dpt, 0, 0, 0);
      }
      uint32_t wq = 0;
      if (DROP) wq = kbits[kbk * Lp + q] >> (4 * h);   // bit 8 g + u: key 8 g + 4 h + u of the block
      bf16x8 sa[2];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 kbv = *(const f32x4*)(kb2 + kbk * 32 + 8 * g + 4 * h);
        ab_p2_pairs<DROP>(st, dpt, 4 * g, kbv, lq, dq, wq >> (8 * g), inv, sa);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8 kt = ab_tr8o(Ks + kbk * 4096 + ks * 2048, off.offT[t][0], off.offT[t][1]);
          dQ[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sa[ks], kt, dQ[t], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) dQo[t][e >> 3][e & 7] = (__bf16)(dQ[t][e] * a.scale);
  }
  __syncthreads();
  // element (row 8 (e >> 2) + 4 h + (e & 3) of block blk, column 32 t + r) into a [Lp][64] image
  auto put = [&](char* img, int blk, const bf16x8 (&v)[2][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = blk * 32 + 8 * (e >> 2) + 4 * h + (e & 3), col = 32 * t + r;
        *(__bf16*)(img + ab_rc(row, col >> 3) + (col & 7) * 2) = v[t][e >> 3][e & 7];
      }
  };
  // dsum: each unit's column sums over its 32 rows (of the values as stored; rows past L are
  // exactly 0) into the V image, dead from here on: [NB][3 (dQ, dK, dV)][64]
  float* csum = (float*)Vs;
  auto colsum32 = [&](int blk, int m, const bf16x8 (&v)[2][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float x = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) x += (float)v[t][e >> 3][e & 7];
      x += __shfl_xor(x, 32, 64);
      if (h == 0) csum[(blk * 3 + m) * 64 + 32 * t + r] = x;
    }
  };
  if (p1 >= 0) {
    put(Qs, p1, dKo);
    put(Os, p1, dVo);
    if (a.dsum) {
      colsum32(p1, 1, dKo);
      colsum32(p1, 2, dVo);
    }
  }
  if (p2 >= 0) {
    put(Ks, p2, dQo);
    if (a.dsum) colsum32(p2, 0, dQo);
  }
  __syncthreads();
  // ---- rows out: dQ (K image), dK (Qs image), dV (dO image), 16 B per lane, 8 lanes per row
#pragma unroll
  for (int it = 0; it < (3 * Lp * 8 + NT - 1) / NT; ++it) {
    const int i = tid + it * NT;
    const int m = i / (Lp * 8), rem = i - m * (Lp * 8);   // m: 0 dQ, 1 dK, 2 dV
    const int row = rem >> 3, c = rem & 7;
    if (m < 3 && row < L) {
      const char* img = m == 0 ? Ks : (m == 1 ? Qs : Os);
      *(bf16x8*)(a.dqkv + (row0 + row) * ld + m * a.H + hd * 64 + c * 8) = *(const bf16x8*)(img + ab_rc(row, c));
    }
  }
  if (a.dsum && tid < 192) {   // the blocks' column sums in block order -> dsum[b][3H]
    const int m = tid >> 6, col = tid & 63;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < NB; ++k) t += csum[(k * 3 + m) * 64 + col];
    a.dsum[b * 3 * (int64_t)a.H + m * a.H + hd * 64 + col] = t;
  }
}

// ---------------------------------------------------------------------------
// Attention backward for 160 < L <= 512 (BERT's max_position_embeddings; the whole-sequence kernel
// above holds Qs, K, V, dO of the sequence in LDS, which stops at 160 rows): the same two phases,
// each as its own kernel over 128-row groups, with the OTHER side streamed through LDS 32 rows at
// a time (FlashAttention-2 style):
//   dkdv: work-group = (sequence, head, 128 keys), wave = 32 keys (K, V fragments in registers);
//         loop over the query blocks: Qs, dO rows (+ Dv from O, lse, keep words) staged in LDS;
//   dq:   work-group = (sequence, head, 128 queries), wave = 32 queries (Qs, dO in registers);
//         loop over the key blocks: K, V rows and the key bias staged in LDS.
// Every score product, exponential and MFMA operand layout is the phase's of
// attention_bwd_rk_kernel (same arithmetic per element).  The next block's global loads are issued
// before the current block's matrix work (one barrier pair per block).  Dropout needs the forward's
// keep bits (drt_attention_train_fwd_bits_bf16).  dsum: column sums per (sequence, 128-row group)
// [B][G][3H], reduced in a fixed order by the caller (deterministic).
// ---------------------------------------------------------------------------
constexpr int kAblMaxSeq = 512;
constexpr int kAblGroup = 128;   // rows per work-group (4 waves x 32)

template <bool DROP>
__global__ __launch_bounds__(256, 2) void attention_bwd_long_dkdv_kernel(AttnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) char Qs[32 * kAbRow];
  __shared__ __attribute__((aligned(16))) char Os[32 * kAbRow];
  __shared__ __attribute__((aligned(16))) float lse2[32];
  __shared__ __attribute__((aligned(16))) float dvs[32];
  __shared__ __attribute__((aligned(16))) uint32_t kw[4][32];
  __shared__ __attribute__((aligned(16))) char Out[2][kAblGroup * kAbRow];   // dK, dV rows out
  __shared__ float csum[4][2][64];
  const int L = (int)a.L;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t b = blockIdx.x / a.heads;
  const int hd = blockIdx.x % a.heads;
  const int grp = blockIdx.y;
  const int64_t row0 = b * a.L;
  const int64_t hrow = ((int64_t)b * a.heads + hd) * a.L;
  const int64_t ld = 3 * (int64_t)a.H;
  const int nkw = (L + 31) >> 5;                     // keep words per query row
  const int nqb = nkw;                               // query blocks
  const __bf16* Qg = a.qkv + row0 * ld + hd * 64;
  const __bf16* Kg = Qg + a.H;
  const __bf16* Vg = Qg + 2 * a.H;
  const __bf16* Og = a.ctx + row0 * a.H + hd * 64;
  const __bf16* dOg = a.dctx + row0 * a.H + hd * 64;
  const int blk = grp * 4 + wave;                    // this wave's key block
  const int key = blk * 32 + r;
  const bool active = blk * 32 < L;                  // wave-uniform
  const int keyc = key < L ? key : L - 1;
  bf16x8 kf[4], vf[4];                               // B operands of S = Qs K^T, dP = dO V^T
#pragma unroll
  for (int k4 = 0; k4 < 4; ++k4) {
    kf[k4] = *(const bf16x8*)(Kg + (int64_t)keyc * ld + (2 * k4 + h) * 8);
    vf[k4] = *(const bf16x8*)(Vg + (int64_t)keyc * ld + (2 * k4 + h) * 8);
    if (key >= L) {
      kf[k4] = bf16x8{};
      vf[k4] = bf16x8{};
    }
  }
  const float kbias = (key >= L || (a.mask && a.mask[b * a.L + key] == 0)) ? -3.402823466e+38f : 0.0f;
  const float inv = DROP ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const AbOffsets off = ab_offsets(lane);
  const uint32_t lanebit = 1u << r;

  // staging of query block qb: thread (row = tid >> 3, chunk c = tid & 7)
  const int srow = tid >> 3, sc = tid & 7;
  bf16x8 gq, go, goo;
  float glse = 0.f;
  uint32_t gw = 0u;
  auto load = [&](int qb) {
    const int q = qb * 32 + srow;
    gq = go = goo = bf16x8{};
    if (q < L) {
      gq = *(const bf16x8*)(Qg + (int64_t)q * ld + sc * 8);
      go = *(const bf16x8*)(dOg + (int64_t)q * a.H + sc * 8);
      goo = *(const bf16x8*)(Og + (int64_t)q * a.H + sc * 8);
    }
    if (tid < 32) glse = qb * 32 + tid < L ? a.lse[hrow + qb * 32 + tid] : 0.f;
    if (DROP && tid < 128) {
      const int w = tid >> 5, qq = qb * 32 + (tid & 31), kb = grp * 4 + w;
      gw = (qq < L && kb < nkw) ? a.drop_bits[(hrow + qq) * nkw + kb] : 0u;
    }
  };
  auto store = [&](int qb) {
    float part = 0.f;
    bf16x8 qv = gq;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      qv[j] = (__bf16)((float)qv[j] * a.scale);
      part += (float)go[j] * (float)goo[j];
    }
    *(bf16x8*)(Qs + ab_rc(srow, sc)) = qv;
    *(bf16x8*)(Os + ab_rc(srow, sc)) = go;
    part += __shfl_xor(part, 1, 64);
    part += __shfl_xor(part, 2, 64);
    part += __shfl_xor(part, 4, 64);
    if (sc == 0) dvs[srow] = part;
    // rows past L: lse2 = +inf makes P = 0 (their dO is 0 too)
    if (tid < 32) lse2[tid] = qb * 32 + tid < L ? glse * kLog2e : __builtin_inff();
    if (DROP && tid < 128) kw[tid >> 5][tid & 31] = gw;
  };

  f32x16 dK[2], dV[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      dK[t][e] = 0.f;
      dV[t][e] = 0.f;
    }
  load(0);
  for (int qb = 0; qb < nqb; ++qb) {
    store(qb);
    __syncthreads();
    if (qb + 1 < nqb) load(qb + 1);   // in flight during this block's matrix work
    if (active) {
      f32x16 sv, dp;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        sv[e] = 0.f;
        dp[e] = 0.f;
      }
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const bf16x8 qa = *(const bf16x8*)(Qs + off.offA[k4]);
        sv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[k4], sv, 0, 0, 0);
        const bf16x8 oa = *(const bf16x8*)(Os + off.offA[k4]);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(oa, vf[k4], dp, 0, 0, 0);
      }
      bf16x8 pa[2], sa[2];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int q0 = 8 * g + 4 * h;
        const f32x4 lq = *(const f32x4*)(lse2 + q0);
        const f32x4 dq = *(const f32x4*)(dvs + q0);
        u32x4 wk = {};
        if (DROP) wk = *(const u32x4*)(&kw[wave][q0]);
        ab_p1_pairs<DROP>(sv, dp, 4 * g, lq, dq, kbias, wk, lanebit, inv, pa, sa);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8 ob = ab_tr8o(Os + ks * 2048, off.offT[t][0], off.offT[t][1]);
          dV[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa[ks], ob, dV[t], 0, 0, 0);
          const bf16x8 qb8 = ab_tr8o(Qs + ks * 2048, off.offT[t][0], off.offT[t][1]);
          dK[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sa[ks], qb8, dK[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // rows out through LDS: element (key row 8 (e >> 2) + 4 h + (e & 3) of the wave's block, column
  // 32 t + r); dsum: the wave's column sums of the stored values, then the 4 waves in order
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float sk = 0.f, sv2 = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = wave * 32 + 8 * (e >> 2) + 4 * h + (e & 3), col = 32 * t + r;
      const __bf16 vk = (__bf16)dK[t][e];
      const __bf16 vv = (__bf16)(DROP ? dV[t][e] * inv : dV[t][e]);
      *(__bf16*)(Out[0] + ab_rc(row, col >> 3) + (col & 7) * 2) = vk;
      *(__bf16*)(Out[1] + ab_rc(row, col >> 3) + (col & 7) * 2) = vv;
      sk += (float)vk;
      sv2 += (float)vv;
    }
    sk += __shfl_xor(sk, 32, 64);
    sv2 += __shfl_xor(sv2, 32, 64);
    if (h == 0) {
      csum[wave][0][32 * t + r] = sk;
      csum[wave][1][32 * t + r] = sv2;
    }
  }
  __syncthreads();
  for (int i = tid; i < kAblGroup * 8; i += 256) {   // 16 B per lane, 8 lanes per row
    const int row = i >> 3, c = i & 7, kk = grp * kAblGroup + row;
    if (kk < L) {
      *(bf16x8*)(a.dqkv + (row0 + kk) * ld + a.H + hd * 64 + c * 8) = *(const bf16x8*)(Out[0] + ab_rc(row, c));
      *(bf16x8*)(a.dqkv + (row0 + kk) * ld + 2 * a.H + hd * 64 + c * 8) = *(const bf16x8*)(Out[1] + ab_rc(row, c));
    }
  }
  if (a.dsum && tid < 128) {   // [B][G][3H]
    const int G = (L + kAblGroup - 1) / kAblGroup;
    const int m = tid >> 6, col = tid & 63;   // m: 0 dK, 1 dV
    a.dsum[((int64_t)b * G + grp) * 3 * a.H + (1 + m) * a.H + hd * 64 + col] =
        csum[0][m][col] + csum[1][m][col] + csum[2][m][col] + csum[3][m][col];
  }
}

template <bool DROP>
__global__ __launch_bounds__(256, 2) void attention_bwd_long_dq_kernel(AttnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) char Ks[32 * kAbRow];
  __shared__ __attribute__((aligned(16))) char Vs[32 * kAbRow];
  __shared__ __attribute__((aligned(16))) float kb2[32];
  __shared__ __attribute__((aligned(16))) char Out[kAblGroup * kAbRow];
  __shared__ float csum[4][64];
  const int L = (int)a.L;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t b = blockIdx.x / a.heads;
  const int hd = blockIdx.x % a.heads;
  const int grp = blockIdx.y;
  const int64_t row0 = b * a.L;
  const int64_t hrow = ((int64_t)b * a.heads + hd) * a.L;
  const int64_t ld = 3 * (int64_t)a.H;
  const int nkw = (L + 31) >> 5;
  const int nkb = nkw;
  const __bf16* Qg = a.qkv + row0 * ld + hd * 64;
  const __bf16* Kg = Qg + a.H;
  const __bf16* Vg = Qg + 2 * a.H;
  const __bf16* Og = a.ctx + row0 * a.H + hd * 64;
  const __bf16* dOg = a.dctx + row0 * a.H + hd * 64;
  const int blk = grp * 4 + wave;
  const int q = blk * 32 + r;                        // this lane's query (D column)
  const bool active = blk * 32 < L;
  const int qc = q < L ? q : L - 1;
  bf16x8 qf[4], of[4];                               // B operands of S^T = K Qs^T, dP^T = V dO^T
  float part = 0.f;
#pragma unroll
  for (int k4 = 0; k4 < 4; ++k4) {
    bf16x8 x = *(const bf16x8*)(Qg + (int64_t)qc * ld + (2 * k4 + h) * 8);
    const bf16x8 o = *(const bf16x8*)(dOg + (int64_t)qc * a.H + (2 * k4 + h) * 8);
    const bf16x8 oo = *(const bf16x8*)(Og + (int64_t)qc * a.H + (2 * k4 + h) * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x[j] = (__bf16)((float)x[j] * a.scale);
      part += (float)o[j] * (float)oo[j];
    }
    qf[k4] = q < L ? x : bf16x8{};
    of[k4] = q < L ? o : bf16x8{};
  }
  part += __shfl_xor(part, 32, 64);                 // Dv over the 64 d (the two lane halves)
  const float dq = part;
  const float lq = q < L ? a.lse[hrow + q] * kLog2e : __builtin_inff();
  const float inv = DROP ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const AbOffsets off = ab_offsets(lane);

  const int srow = tid >> 3, sc = tid & 7;
  bf16x8 gk, gv;
  float gkb = 0.f;
  uint32_t gw = 0u;
  auto load = [&](int kb) {
    const int kk = kb * 32 + srow;
    gk = gv = bf16x8{};
    if (kk < L) {
      gk = *(const bf16x8*)(Kg + (int64_t)kk * ld + sc * 8);
      gv = *(const bf16x8*)(Vg + (int64_t)kk * ld + sc * 8);
    }
    if (tid < 32) {
      const int k2 = kb * 32 + tid;
      gkb = (k2 >= L || (a.mask && a.mask[b * a.L + k2] == 0)) ? -3.402823466e+38f : 0.0f;
    }
    if (DROP) gw = q < L ? a.drop_bits[(hrow + q) * nkw + kb] : 0u;
  };
  auto store = [&]() {
    *(bf16x8*)(Ks + ab_rc(srow, sc)) = gk;
    *(bf16x8*)(Vs + ab_rc(srow, sc)) = gv;
    if (tid < 32) kb2[tid] = gkb;
  };
  f32x16 dQ[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) dQ[t][e] = 0.f;
  load(0);
  for (int kb = 0; kb < nkb; ++kb) {
    store();
    const uint32_t wq0 = DROP ? gw >> (4 * h) : 0u;   // bit 8 g + u: key 8 g + 4 h + u of the block
    __syncthreads();
    if (kb + 1 < nkb) load(kb + 1);
    if (active) {
      f32x16 st, dpt;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        st[e] = 0.f;
        dpt[e] = 0.f;
      }
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const bf16x8 ka = *(const bf16x8*)(Ks + off.offA[k4]);
        st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[k4], st, 0, 0, 0);
        const bf16x8 va = *(const bf16x8*)(Vs + off.offA[k4]);
        dpt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, of[k4], dpt, 0, 0, 0);
      }
      bf16x8 sa[2];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 kbv = *(const f32x4*)(kb2 + 8 * g + 4 * h);
        ab_p2_pairs<DROP>(st, dpt, 4 * g, kbv, lq, dq, wq0 >> (8 * g), inv, sa);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8 kt = ab_tr8o(Ks + ks * 2048, off.offT[t][0], off.offT[t][1]);
          dQ[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sa[ks], kt, dQ[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // rows out: element (query row 8 (e >> 2) + 4 h + (e & 3) of the wave's block, column 32 t + r)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float sq = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = wave * 32 + 8 * (e >> 2) + 4 * h + (e & 3), col = 32 * t + r;
      const __bf16 v = (__bf16)(dQ[t][e] * a.scale);
      *(__bf16*)(Out + ab_rc(row, col >> 3) + (col & 7) * 2) = v;
      sq += (float)v;
    }
    sq += __shfl_xor(sq, 32, 64);
    if (h == 0) csum[wave][32 * t + r] = sq;
  }
  __syncthreads();
  for (int i = tid; i < kAblGroup * 8; i += 256) {
    const int row = i >> 3, c = i & 7, qq = grp * kAblGroup + row;
    if (qq < L) *(bf16x8*)(a.dqkv + (row0 + qq) * ld + hd * 64 + c * 8) = *(const bf16x8*)(Out + ab_rc(row, c));
  }
  if (a.dsum && tid < 64) {
    const int G = (L + kAblGroup - 1) / kAblGroup;
    a.dsum[((int64_t)b * G + grp) * 3 * a.H + hd * 64 + tid] = csum[0][tid] + csum[1][tid] + csum[2][tid] + csum[3][tid];
  }
}

// out = dropout(y) (+ resid): keep iff drop_hash24(seed, site, i) >= p 2^24, kept values scaled
// by 1 / (1 - p).  The same call on a gradient (resid = NULL) is the dropout backward.
__global__ __launch_bounds__(256) void dropout_add_kernel(const __bf16* y, const __bf16* resid, int64_t n, float p,
                                                          uint64_t seed, uint64_t site, __bf16* out) {
  const int64_t i8 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i8 >= n) return;
  const uint32_t thr = drop_threshold(p);
  const float inv = 1.0f / (1.0f - p);
  if (i8 + 8 <= n) {   // 16-B pieces
    const bf16x8 yv = *(const bf16x8*)(y + i8);
    bf16x8 rv = {};
    if (resid) rv = *(const bf16x8*)(resid + i8);
    bf16x8 o;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool keep = drop_hash24(seed, site, (uint64_t)(i8 + u)) >= thr;
      float v = keep ? (float)yv[u] * inv : 0.0f;
      if (resid) v += (float)rv[u];
      o[u] = (__bf16)v;
    }
    *(bf16x8*)(out + i8) = o;
  } else {
    for (int64_t i = i8; i < n; ++i) {
      const bool keep = drop_hash24(seed, site, (uint64_t)i) >= thr;
      float v = keep ? (float)y[i] * inv : 0.0f;
      if (resid) v += (float)resid[i];
      out[i] = (__bf16)v;
    }
  }
}

// Row slabs of the first colsum pass: enough blocks to fill the chip (~1024 with the column
// blocks of 512 bf16 columns), >= 64 rows per slab (16 per wave), <= 512 slabs (the second pass,
// 256 fp32 columns per block, sums them in order).
static int64_t colsum_slabs(int64_t M, int64_t N) {
  if (M < 256) return 1;
  const int64_t gx = (N + 511) / 512;
  int64_t slabs = (1024 + gx - 1) / gx;
  if (slabs > M / 64) slabs = M / 64;
  if (slabs > 512) slabs = 512;
  return slabs < 1 ? 1 : slabs;
}

template <typename T>
static unsigned colsum_gx(int64_t N) {
  const int64_t cols = 64 * (16 / (int64_t)sizeof(T));
  return (unsigned)((N + cols - 1) / cols);
}

template <typename T>
static int colsum_launch(const T* x, int64_t M, int64_t N, float* out, float* ws, hipStream_t s) {
  const int64_t slabs = colsum_slabs(M, N);
  const int64_t rows_per = (M + slabs - 1) / slabs;
  if (slabs == 1) {
    hipLaunchKernelGGL(colsum_kernel<T>, dim3(colsum_gx<T>(N), 1), dim3(256), 0, s, x, M, N, M, out);
  } else {
    hipLaunchKernelGGL(colsum_kernel<T>, dim3(colsum_gx<T>(N), (unsigned)slabs), dim3(256), 0, s, x, M, N, rows_per,
                       ws);
    hipLaunchKernelGGL(colsum_kernel<float>, dim3(colsum_gx<float>(N), 1), dim3(256), 0, s, (const float*)ws, slabs, N,
                       slabs, out);
  }
  return hip_status(hipGetLastError());
}

}  // namespace drt

using namespace drt;

extern "C" {

size_t drt_colsum_workspace(int64_t M, int64_t N) {
  if (M <= 0 || N <= 0) return 0;
  const int64_t slabs = colsum_slabs(M, N);
  return slabs > 1 ? (size_t)slabs * (size_t)N * sizeof(float) : 0;
}

int drt_colsum_f32(const float* x, int64_t M, int64_t N, float* out, void* ws, size_t ws_bytes, void* stream) {
  DRT_REQUIRE(M >= 0 && N >= 0);
  if (N == 0) return DRT_OK;
  DRT_REQUIRE(out);
  hipStream_t s = (hipStream_t)stream;
  if (M == 0) return hip_status(hipMemsetAsync(out, 0, N * sizeof(float), s));
  DRT_REQUIRE(x && ws_bytes >= drt_colsum_workspace(M, N) && (ws || drt_colsum_workspace(M, N) == 0));
  return colsum_launch<float>(x, M, N, out, (float*)ws, s);
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
  return (size_t)3 * kLnBwdBlocks * (size_t)H * sizeof(float) + drt_colsum_workspace(kLnBwdBlocks, 2 * H);
}

// dx = LN backward of dy through out = LN(x) (gamma; x = the bf16 pre-LN sums the forward
// stored) + dres (residual gradient, may be NULL); dgamma / dbeta fp32 [H] (deterministic).
int drt_layernorm_bwd_drop_bf16(const void* dy, const void* x, const float* gamma, float eps, int64_t M, int32_t H,
                                const void* dres, void* dx, void* dx_drop, float drop_p, uint64_t seed, uint64_t site,
                                float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream);

int drt_layernorm_bwd_bf16(const void* dy, const void* x, const float* gamma, float eps, int64_t M, int32_t H,
                           const void* dres, void* dx, float* dgamma, float* dbeta, void* ws, size_t ws_bytes,
                           void* stream) {
  return drt_layernorm_bwd_drop_bf16(dy, x, gamma, eps, M, H, dres, dx, nullptr, 0.f, 0, 0, dgamma, dbeta, ws,
                                     ws_bytes, stream);
}

int drt_layernorm_bwd_sum_bf16(const void* dy, const void* x, const float* gamma, float eps, int64_t M, int32_t H,
                               const void* dres, void* dx, void* dx_drop, float drop_p, uint64_t seed, uint64_t site,
                               float* dgamma, float* dbeta, float* dsum, void* ws, size_t ws_bytes, void* stream);

// The same, also writing dx_drop = dropout(dx) with drt_dropout_add_bf16's mask of (drop_p, seed, site)
// (the gradient entering the linear whose output HF dropped before this LayerNorm's residual add).
int drt_layernorm_bwd_drop_bf16(const void* dy, const void* x, const float* gamma, float eps, int64_t M, int32_t H,
                                const void* dres, void* dx, void* dx_drop, float drop_p, uint64_t seed, uint64_t site,
                                float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream) {
  return drt_layernorm_bwd_sum_bf16(dy, x, gamma, eps, M, H, dres, dx, dx_drop, drop_p, seed, site, dgamma, dbeta,
                                    nullptr, ws, ws_bytes, stream);
}

// The same, also writing dsum [H] fp32 = the column sums of the gradient it hands down (dx_drop,
// or dx without dropout) -- the bias gradient of the linear feeding this LayerNorm.
int drt_layernorm_bwd_sum_bf16(const void* dy, const void* x, const float* gamma, float eps, int64_t M, int32_t H,
                               const void* dres, void* dx, void* dx_drop, float drop_p, uint64_t seed, uint64_t site,
                               float* dgamma, float* dbeta, float* dsum, void* ws, size_t ws_bytes, void* stream) {
  DRT_REQUIRE(M > 0 && H > 0 && H % 256 == 0 && H <= 1024);
  DRT_REQUIRE(!dx_drop || (drop_p >= 0.f && drop_p < 1.f));
  DRT_REQUIRE(dy && x && gamma && dx && dgamma && dbeta && ws && ws_bytes >= drt_layernorm_bwd_workspace(M, H));
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)ws;   // [3 * blocks][H]: dgamma rows, dbeta rows, dsum rows
  const dim3 grid(kLnBwdBlocks);
#define LNB(E, S)                                                                                                   \
  hipLaunchKernelGGL((layernorm_bwd_kernel<E, S>), grid, dim3(256), 0, s, (const __bf16*)dy, (const __bf16*)x, gamma, \
                     eps, M, (int)H, (const __bf16*)dres, (__bf16*)dx, part, (__bf16*)dx_drop, drop_p, seed, site)
#define LNB2(E) \
  if (dsum) LNB(E, true); \
  else LNB(E, false);
  switch (H / 64) {
    case 4: LNB2(4); break;
    case 8: LNB2(8); break;
    case 12: LNB2(12); break;
    case 16: LNB2(16); break;
    default: return DRT_EINVAL;
  }
#undef LNB2
#undef LNB
  float* ws2 = part + (size_t)3 * kLnBwdBlocks * H;
  int rc = colsum_launch<float>(part, kLnBwdBlocks, H, dgamma, ws2, s);
  if (rc) return rc;
  rc = colsum_launch<float>(part + (size_t)kLnBwdBlocks * H, kLnBwdBlocks, H, dbeta, ws2, s);
  if (rc || !dsum) return rc;
  return colsum_launch<float>(part + (size_t)2 * kLnBwdBlocks * H, kLnBwdBlocks, H, dsum, ws2, s);
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

// dqkv [B*L][3H] (dQ | dK | dV, head-major like qkv) of the attention forward
// (drt_attention_fwd_lse_bf16) given dctx = dO, the forward's ctx = O and lse.  L <= 160.
int drt_attention_train_bwd_bf16(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                                 const int64_t* mask, void* dqkv, int64_t B, int64_t L, int32_t heads,
                                 int32_t head_dim, float scale, float drop_p, uint64_t seed, uint64_t site,
                                 void* stream);

int drt_attention_bwd_bf16(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                           const int64_t* mask, void* dqkv, int64_t B, int64_t L, int32_t heads, int32_t head_dim,
                           float scale, void* stream) {
  return drt_attention_train_bwd_bf16(qkv, ctx, dctx, lse, mask, dqkv, B, L, heads, head_dim, scale, 0.0f, 0, 0,
                                      stream);
}

// The same with the forward's attention-probability dropout (drop_p, seed, site as passed to
// drt_attention_train_fwd_bf16).
int drt_attention_train_bwd_bits_bf16(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                                      const int64_t* mask, const uint32_t* drop_bits, void* dqkv, int64_t B, int64_t L,
                                      int32_t heads, int32_t head_dim, float scale, float drop_p, uint64_t seed,
                                      uint64_t site, void* stream);

int drt_attention_train_bwd_bf16(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                                 const int64_t* mask, void* dqkv, int64_t B, int64_t L, int32_t heads,
                                 int32_t head_dim, float scale, float drop_p, uint64_t seed, uint64_t site,
                                 void* stream) {
  return drt_attention_train_bwd_bits_bf16(qkv, ctx, dctx, lse, mask, nullptr, dqkv, B, L, heads, head_dim, scale,
                                           drop_p, seed, site, stream);
}

// The same reading the forward's keep bits (drt_attention_train_fwd_bits_bf16) instead of re-hashing
// every (query, key) twice (dK / dV and dQ phases); NULL drop_bits = regenerate from the hash.
static int attention_bwd_launch(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                                const int64_t* mask, const uint32_t* drop_bits, void* dqkv, int64_t B, int64_t L,
                                int32_t heads, int32_t head_dim, float scale, float drop_p, uint64_t seed,
                                uint64_t site, float* dsum_part, void* stream);

int drt_attention_train_bwd_bits_bf16(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                                      const int64_t* mask, const uint32_t* drop_bits, void* dqkv, int64_t B, int64_t L,
                                      int32_t heads, int32_t head_dim, float scale, float drop_p, uint64_t seed,
                                      uint64_t site, void* stream) {
  return attention_bwd_launch(qkv, ctx, dctx, lse, mask, drop_bits, dqkv, B, L, heads, head_dim, scale, drop_p, seed,
                              site, nullptr, stream);
}

// Sized for any L <= 512: per-(sequence, 128-row group) partials [B][G <= 4][3H] + the colsum's own.
size_t drt_attention_train_bwd_bias_workspace(int64_t B, int32_t heads, int32_t head_dim) {
  if (B <= 0 || heads <= 0 || head_dim <= 0) return 0;
  const int64_t n = 3 * (int64_t)heads * head_dim;
  const int64_t gmax = kAblMaxSeq / kAblGroup;
  return (size_t)B * gmax * n * sizeof(float) + drt_colsum_workspace(B * gmax, n);
}

// The same, also writing dbias [3H] fp32 = the column sums of dQKV (the query / key / value
// bias gradients) from per-sequence (L > 160: per 128-row group) partials the kernels leave in ws,
// reduced in a fixed order -- no pass over dQKV.
int drt_attention_train_bwd_bias_bf16(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                                      const int64_t* mask, const uint32_t* drop_bits, void* dqkv, int64_t B, int64_t L,
                                      int32_t heads, int32_t head_dim, float scale, float drop_p, uint64_t seed,
                                      uint64_t site, float* dbias, void* ws, size_t ws_bytes, void* stream) {
  DRT_REQUIRE(dbias && B > 0 && ws && ws_bytes >= drt_attention_train_bwd_bias_workspace(B, heads, head_dim));
  float* part = (float*)ws;
  int rc = attention_bwd_launch(qkv, ctx, dctx, lse, mask, drop_bits, dqkv, B, L, heads, head_dim, scale, drop_p,
                                seed, site, part, stream);
  if (rc) return rc;
  const int64_t n = 3 * (int64_t)heads * head_dim;
  const int64_t rows = L > kAbMaxSeq ? B * ((L + kAblGroup - 1) / kAblGroup) : B;
  const int64_t gmax = kAblMaxSeq / kAblGroup;
  return colsum_launch<float>(part, rows, n, dbias, part + (size_t)B * gmax * n, (hipStream_t)stream);
}

static int attention_bwd_launch(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                                const int64_t* mask, const uint32_t* drop_bits, void* dqkv, int64_t B, int64_t L,
                                int32_t heads, int32_t head_dim, float scale, float drop_p, uint64_t seed,
                                uint64_t site, float* dsum_part, void* stream) {
  DRT_REQUIRE(B >= 0 && L > 0 && L <= kAblMaxSeq && heads > 0 && head_dim == 64);
  DRT_REQUIRE(drop_p >= 0.0f && drop_p < 1.0f);
  if (B == 0) return DRT_OK;
  DRT_REQUIRE(qkv && ctx && dctx && lse && dqkv);
  AttnBwdArgs a{(const __bf16*)qkv, (const __bf16*)ctx, (const __bf16*)dctx, lse, mask, (__bf16*)dqkv, B, L,
                heads, heads * 64, scale, drop_p, seed, site, drop_bits, dsum_part};
  if (L > kAbMaxSeq) {   // streamed kernels: dK / dV over key groups, dQ over query groups
    const bool drop = drop_p > 0.0f;
    DRT_REQUIRE(!drop || drop_bits);   // the forward's keep bits (drt_attention_train_fwd_bits_bf16)
    const dim3 grid((unsigned)(B * heads), (unsigned)((L + kAblGroup - 1) / kAblGroup));
    hipStream_t st = (hipStream_t)stream;
    if (drop) {
      hipLaunchKernelGGL((attention_bwd_long_dkdv_kernel<true>), grid, dim3(256), 0, st, a);
      hipLaunchKernelGGL((attention_bwd_long_dq_kernel<true>), grid, dim3(256), 0, st, a);
    } else {
      hipLaunchKernelGGL((attention_bwd_long_dkdv_kernel<false>), grid, dim3(256), 0, st, a);
      hipLaunchKernelGGL((attention_bwd_long_dq_kernel<false>), grid, dim3(256), 0, st, a);
    }
    return hip_status(hipGetLastError());
  }
  const int Lp = ((int)L + 31) & ~31;
  const int nb = Lp / 32;
  const dim3 grid((unsigned)(B * heads));
  const bool drop = drop_p > 0.0f;
  // register-resident P / dS; dropout from the forward's keep bits (or the same bits drawn again)
  size_t lds = (size_t)4 * Lp * kAbRow + (size_t)3 * Lp * 4 + (drop ? (size_t)nb * Lp * 4 : 0);
  DRT_REQUIRE(lds <= 160 * 1024);
  static bool rk_attr = false;
  if (!rk_attr) {
    const void* ks[] = {(const void*)attention_bwd_rk_kernel<4, false>, (const void*)attention_bwd_rk_kernel<4, true>,
                        (const void*)attention_bwd_rk_kernel<5, false>, (const void*)attention_bwd_rk_kernel<5, true>};
    for (const void* f : ks) DRT_CHECK_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    rk_attr = true;
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 blk(nb == 5 ? 512 : 256);
#define DRT_AB_LAUNCH(NB_)                                                                              \
  case NB_:                                                                                             \
    if (drop) hipLaunchKernelGGL((attention_bwd_rk_kernel<NB_, true>), grid, blk, lds, st, a);         \
    else hipLaunchKernelGGL((attention_bwd_rk_kernel<NB_, false>), grid, blk, lds, st, a);             \
    break;
  switch (nb) {
    DRT_AB_LAUNCH(1)
    DRT_AB_LAUNCH(2)
    DRT_AB_LAUNCH(3)
    DRT_AB_LAUNCH(4)
    DRT_AB_LAUNCH(5)
    default: return DRT_EINVAL;
  }
#undef DRT_AB_LAUNCH
  return hip_status(hipGetLastError());
}

int drt_dropout_add_bf16(const void* y, const void* resid, int64_t n, float p, uint64_t seed, uint64_t site,
                         void* out, void* stream) {
  DRT_REQUIRE(n >= 0 && p >= 0.0f && p < 1.0f);
  if (n == 0) return DRT_OK;
  DRT_REQUIRE(y && out);
  DRT_REQUIRE((uintptr_t)y % 16 == 0 && (uintptr_t)out % 16 == 0 && (!resid || (uintptr_t)resid % 16 == 0));
  hipLaunchKernelGGL(dropout_add_kernel, dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)y, (const __bf16*)resid, n, p, seed, site, (__bf16*)out);
  return hip_status(hipGetLastError());
}

int drt_transpose_bf16_ld(const void* x, int64_t R, int64_t C, void* y, int64_t ldy, void* stream) {
  DRT_REQUIRE(R >= 0 && C >= 0 && ldy >= R);
  if (R == 0 || C == 0) return DRT_OK;
  DRT_REQUIRE(x && y && ((uintptr_t)x % 16 == 0) && ((uintptr_t)y % 16 == 0));
  dim3 grid((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64));
  hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const __bf16*)x, R, C,
                     (__bf16*)y, ldy);
  return hip_status(hipGetLastError());
}

int drt_transpose_bf16(const void* x, int64_t R, int64_t C, void* y, void* stream) {
  return drt_transpose_bf16_ld(x, R, C, y, R, stream);
}

}  // extern "C"
