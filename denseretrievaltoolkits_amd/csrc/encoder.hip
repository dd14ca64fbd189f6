// BERT bi-encoder forward kernels (DRModel.encode, DRT/model/biencoder.py:127-151,
// over HF BertModel: transformers/models/bert/modeling_bert.py embeddings :53-107,
// self-attention :139-204, sublayer outputs :282-352).
//
//   embed_ln        word + position + token-type embedding, LayerNorm (fp32 math)
//   layernorm       LayerNorm of an fp32 [M, H] row (GEMM epilogue already added
//                   bias + residual), bf16 out
//   attention       per (sequence, head): softmax(Q K^T / sqrt(dh) + key mask) V
//                   with v_mfma_f32_32x32x16_bf16, online softmax over 32-key
//                   tiles; S^T = K Q^T keeps each query's scores lane-local and
//                   the S^T accumulator feeds the P.V MFMA directly as its B
//                   operand (no LDS round trip for P)
//   pool            first / masked-mean / masked-max pooling (utils.py:233-240)
//   l2norm          F.normalize(reps, dim=1) (biencoder.py:149-150)
#include "drt_common.h"
#include "ln_row.h"

namespace drt {

template <int EPL>
__global__ __launch_bounds__(256) void embed_ln_kernel(const int64_t* ids, const int64_t* type_ids, int64_t T,
                                                       int64_t L, const float* wemb, const float* pemb,
                                                       const float* temb, const float* gamma, const float* beta,
                                                       float eps, int H, __bf16* out, __bf16* pre = nullptr) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const int64_t id = ids[t];
  const int64_t pos = t % L;
  const int64_t tt = type_ids ? type_ids[t] : 0;
  const float* w = wemb + id * H;
  const float* p = pemb + pos * H;
  const float* y = temb + tt * H;
  float x[EPL];
#pragma unroll
  for (int e4 = 0; e4 < EPL / 4; ++e4) {
    const int c = e4 * 256 + lane * 4;
    const f32x4 a = *(const f32x4*)(w + c);
    const f32x4 b = *(const f32x4*)(p + c);
    const f32x4 d = *(const f32x4*)(y + c);
#pragma unroll
    for (int u = 0; u < 4; ++u) x[e4 * 4 + u] = (a[u] + d[u]) + b[u];  // (word + type) + position, as HF
    if (pre) {   // training forward: the pre-LN sum, input of the LayerNorm backward
      bf16x4 o;
#pragma unroll
      for (int u = 0; u < 4; ++u) o[u] = (__bf16)x[e4 * 4 + u];
      *(bf16x4*)(pre + t * H + c) = o;
    }
  }
  ln_row<EPL>(x, gamma, beta, eps, lane, H, out + t * H);
}

// erf GELU, elementwise (the training forward keeps FFN1's pre-activation for the backward)
__global__ __launch_bounds__(256) void gelu_kernel(const __bf16* x, int64_t n, __bf16* y) {
  const int64_t i8 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i8 >= n) return;
  if (i8 + 8 <= n) {   // 16-B pieces
    const bf16x8 xv = *(const bf16x8*)(x + i8);
    bf16x8 o;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float v = (float)xv[u];
      o[u] = (__bf16)(0.5f * v * (1.0f + erff(v * 0.70710678118654752f)));
    }
    *(bf16x8*)(y + i8) = o;
  } else {
    for (int64_t i = i8; i < n; ++i) {
      const float v = (float)x[i];
      y[i] = (__bf16)(0.5f * v * (1.0f + erff(v * 0.70710678118654752f)));
    }
  }
}

// Embedding backward (BertEmbeddings, modeling_bert.py:68-108): the gradient of the pre-LN sum
// goes to the word / position / token-type tables (fp32, caller zeroes them).
// Word rows: one block per token, fp32 atomics (the row ids are spread over the vocabulary).
__global__ __launch_bounds__(256) void embedding_bwd_word_kernel(const int64_t* ids, const __bf16* d, int H,
                                                                 int64_t padding_idx, float* dword) {
  const int64_t t = (int64_t)blockIdx.x;
  const int64_t id = ids[t];
  if (id == padding_idx) return;   // nn.Embedding(padding_idx): the row stays 0
  for (int c = threadIdx.x; c < H; c += 256) atomicAdd(dword + id * H + c, (float)d[t * H + c]);
}

// Token-type rows with type ids (BERT: 2 rows, every token adds to one of them -- per-token atomics
// were T-way contended): a block sums one column slab over a chunk of kTypeChunk tokens per type
// in registers and adds once per (chunk, element).  Grid (column slabs, token chunks).
constexpr int kTypeChunk = 1024;
constexpr int kMaxTypes = 4;
__global__ __launch_bounds__(256) void embedding_bwd_type_kernel(const int64_t* type_ids, const __bf16* d, int64_t T,
                                                                 int H, int ntypes, float* dtype) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= H) return;
  const int64_t t0 = (int64_t)blockIdx.y * kTypeChunk;
  const int64_t t1 = t0 + kTypeChunk < T ? t0 + kTypeChunk : T;
  float s[kMaxTypes] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t t = t0; t < t1; ++t) {
    const int64_t tt = type_ids[t];
    const float g = (float)d[t * H + c];
#pragma unroll
    for (int y = 0; y < kMaxTypes; ++y) s[y] += tt == y ? g : 0.0f;
  }
#pragma unroll
  for (int y = 0; y < kMaxTypes; ++y)
    if (y < ntypes && s[y] != 0.0f) atomicAdd(dtype + (int64_t)y * H + c, s[y]);
}

// Position rows: every sequence adds to rows 0..L-1, so per-element atomics from every token were
// B-way contended (and the single token-type row T-way: 2.1 ms per passage tower at B 1024, L 128).
// Here a block sums a chunk of kPosChunk sequences for one position and column slab in registers
// and adds once (B / kPosChunk atomics per element).
constexpr int kPosChunk = 64;
__global__ __launch_bounds__(256) void embedding_bwd_pos_kernel(const __bf16* d, int64_t B, int64_t L, int H,
                                                                float* dpos) {
  const int64_t p = blockIdx.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= H) return;
  const int64_t b0 = (int64_t)blockIdx.z * kPosChunk;
  const int64_t b1 = b0 + kPosChunk < B ? b0 + kPosChunk : B;
  float s = 0.f;
  for (int64_t b = b0; b < b1; ++b) s += (float)d[(b * L + p) * H + c];
  atomicAdd(dpos + p * H + c, s);
}

// Token type 0 without type ids: every token adds to row 0, i.e. dtype[0] += sum of the rows
// dpos[0..L-1] this call produced (dpos arrives zeroed).
__global__ __launch_bounds__(256) void embedding_bwd_type0_kernel(const float* dpos, int64_t L, int H, float* dtype) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= H) return;
  float s = 0.f;
  for (int64_t p = 0; p < L; ++p) s += dpos[p * H + c];
  dtype[c] += s;
}

template <int EPL>
__global__ __launch_bounds__(256) void layernorm_f32_kernel(const float* X, int64_t M, int H, const float* gamma,
                                                            const float* beta, float eps, __bf16* out) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= M) return;
  const float* xr = X + t * H;
  float x[EPL];
#pragma unroll
  for (int e4 = 0; e4 < EPL / 4; ++e4) {
    const f32x4 a = *(const f32x4*)(xr + e4 * 256 + lane * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) x[e4 * 4 + u] = a[u];
  }
  ln_row<EPL>(x, gamma, beta, eps, lane, H, out + t * H);
}

// Same LayerNorm over bf16 pre-LN sums (the encoder's default: the GEMM epilogue
// adds bias + residual in fp32 and rounds once, halving the bytes of both sides).
// Round 6: one round of work-groups, each wave normalising rows t, t + waves, ... with gamma / beta
// held in registers (loaded once per wave instead of once per row: 2 x EPL / 4 16-B loads per row
// were twice the row's own loads through the vector memory pipe) and the next row's loads issued
// before the current row's reductions.  Same per-row arithmetic (ln_row_gb): bit-identical.
template <int EPL>
__global__ __launch_bounds__(256) void layernorm_bf16_kernel(const __bf16* X, int64_t M, int H, const float* gamma,
                                                             const float* beta, float eps, __bf16* out) {
  const int lane = threadIdx.x & 63;
  const int64_t t0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  if (t0 >= M) return;
  float g[EPL], b[EPL];
#pragma unroll
  for (int e4 = 0; e4 < EPL / 4; ++e4) {
    const f32x4 gv = *(const f32x4*)(gamma + e4 * 256 + lane * 4);
    const f32x4 bv = *(const f32x4*)(beta + e4 * 256 + lane * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      g[e4 * 4 + u] = gv[u];
      b[e4 * 4 + u] = bv[u];
    }
  }
  bf16x4 cur[EPL / 4];
#pragma unroll
  for (int e4 = 0; e4 < EPL / 4; ++e4) cur[e4] = *(const bf16x4*)(X + t0 * H + e4 * 256 + lane * 4);
  for (int64_t t = t0; t < M; t += nw) {
    const int64_t tn = t + nw;
    bf16x4 nxt[EPL / 4];
    if (tn < M) {
#pragma unroll
      for (int e4 = 0; e4 < EPL / 4; ++e4) nxt[e4] = *(const bf16x4*)(X + tn * H + e4 * 256 + lane * 4);
    }
    float x[EPL];
#pragma unroll
    for (int e4 = 0; e4 < EPL / 4; ++e4)
#pragma unroll
      for (int u = 0; u < 4; ++u) x[e4 * 4 + u] = (float)cur[e4][u];
    ln_row_gb<EPL>(x, g, b, eps, lane, H, out + t * H);
#pragma unroll
    for (int e4 = 0; e4 < EPL / 4; ++e4) cur[e4] = nxt[e4];
  }
}

// Work-groups of the row-looping LayerNorm: 8 per CU (32 waves), at most one per 4 rows.
static unsigned ln_rows_grid(int64_t M) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, v = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
              ? v
              : 256;
  }
  const int64_t need = (M + 3) / 4, cap = (int64_t)cus * 8;
  return (unsigned)(need < cap ? need : cap);
}

// ---------------------------------------------------------------------------
// Attention.  One work-group (4 waves) per (sequence b, head hd); wave w owns
// query blocks w, w+4, ... of 32 rows.  K is staged in LDS as swizzled
// [key][8 x 16 B] rows (A operand of S^T = K Q^T), V transposed as Vt[d][key]
// with a padded row stride (A operand of O^T = V^T P^T).
// ---------------------------------------------------------------------------
constexpr int kAttnThreads = 256;
constexpr int kHeadDim = 64;
constexpr int kMaxSeq = 512;

struct AttnArgs {
  const __bf16* qkv;      // [B*L][3*H]  (Q | K | V, head-major inside each)
  const int64_t* mask;    // [B][L] attention_mask (1 = token, 0 = pad) or null
  __bf16* ctx;            // [B*L][H]
  int64_t B, L;
  int heads, H;
  float scale;            // 1/sqrt(dh): applied to Q (exact for dh = 64)
  float* lse;             // optional [B][heads][L]: log-sum-exp of each query's scaled, masked
                          // scores (what the attention backward needs to rebuild P)
  float drop_p;           // training: dropout of the attention probabilities (DROP kernels)
  uint64_t seed, site;    //   keep = attn_keep(attn_row_key(seed, site, (b * heads + head) * L + q), key)
  uint32_t* drop_bits;    // optional [B][heads][L][ceil(L / 32)]: the keep mask, bit (key & 31) of word
                          //   (query, key >> 5) -- the backward reads it instead of re-hashing
};

// Attention forward, one work-group per (sequence, head): K (swizzled rows), V^T and the key bias
// in LDS, one 32-query block per wave (S^T tiles of 32 keys: rows = keys, lane = query), online
// softmax in registers, P as the B operand of O^T += V^T P^T.  NB = blocks of 32 (Lp = 32 NB) as a
// template argument for L <= 160 (every LDS offset a per-lane constant + an immediate, key loop
// unrolled, O leaves through LDS as whole-row 16-B stores); NB = 0: any L <= 512 (inference), a
// wave loops over its query blocks and stores directly.
// Round 3: scores in log2 units, s2 = fma(s, log2e, kb) with the key bias kb = 0 / -FLT_MAX (finite:
// a row with every key masked gets HF's uniform softmax, no NaN); the running max moves only when a
// tile's max exceeds it by more than kLazy (= 8, P <= 2^8 in bf16 / fp32 is exact to the same
// relative precision), so the O rescale is a rare wave-uniform branch instead of 32 multiplies per
// tile; dropout draws the keep decisions from the pairwise hash (drt_common.h), zeroes dropped P,
// writes the keep words for the backward when asked (drop_bits), and moves 1 / (1 - p) into the
// final 1 / l.  (Drawing the words in a separate one-thread-per-word pass for the forward to read
// measured slower: 272 vs 178 us at 1024 x 128, profiles/r03r_attn_probe.log "bits" vs "hash".)
// lse = (m + log2 l) ln 2 (natural log, what the backward rebuilds P from).
// NW waves: 4, or 5 for 5 query blocks (129 <= L <= 160: the recipe's 156-token passages, the
// reranker's 160-token pairs; with 4, wave 0 ran two blocks while three idled).
constexpr float kLazy = 8.0f;
constexpr float kLn2 = 0.6931471805599453f;

// Register budget: 4 waves per SIMD (<= 128 VGPRs) -- at 5 query blocks the LDS (42 KiB) admits 3
// work-groups of 5 waves per CU, i.e. 4 waves on three of the SIMDs.
template <int NB, bool DROP>
__global__ __launch_bounds__(NB == 5 ? 320 : 256) __attribute__((amdgpu_waves_per_eu(4, 8)))
void attention_fwd_kernel(AttnArgs a) {
  constexpr int NW = NB == 5 ? 5 : 4;
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int L = (int)a.L;
  const int Lp = NB ? NB * 32 : (L + 31) & ~31;  // keys padded to the 32-key tile
  const int nqb = Lp / 32;
  const int vts = Lp * 2 + 8;              // Vt row stride (bytes): conflict-free ds_read_b64
  char* Ks = smem;                          // Lp * 128 B
  char* Vt = smem + Lp * 128;               // 64 * vts B
  float* kb = (float*)(Vt + 64 * vts);      // Lp floats

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t b = blockIdx.x / a.heads;
  const int hd = blockIdx.x % a.heads;
  const int64_t row0 = b * a.L;
  const int64_t hrow = ((int64_t)b * a.heads + hd) * L;
  const int64_t ld = 3 * (int64_t)a.H;
  const __bf16* Qg = a.qkv + row0 * ld + hd * kHeadDim;
  const __bf16* Kg = Qg + a.H;
  const __bf16* Vg = Qg + 2 * a.H;

  // ---- stage K (swizzled rows) and V^T, key bias.  Passes of NT / 2 keys: thread (key group
  // kg = tid >> 3, 16-B chunk c = tid & 7) owns keys 4 kg .. 4 kg + 3 of chunk c, issues all 8
  // global loads of the pass before any LDS store, and writes V^T as 8 ds_write_b64 (4 keys
  // of one d per store) instead of 32 ds_write_b16.  The first Q block's fragments are
  // requested before the pass so their latency overlaps the staging.
  const int c8 = tid & 7, kg = tid >> 3;
  int qrow0 = wave * 32 + (lane & 31);
  qrow0 = qrow0 < L ? qrow0 : L - 1;
  bf16x8 q0[4];
#pragma unroll
  for (int st = 0; st < 4; ++st) q0[st] = *(const bf16x8*)(Qg + (int64_t)qrow0 * ld + st * 16 + (lane >> 5) * 8);
  for (int kp = 0; kp < Lp; kp += NT / 2) {
    u32x4 kv[4], vv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int key = kp + kg * 4 + u;
      kv[u] = u32x4{0u, 0u, 0u, 0u};
      vv[u] = u32x4{0u, 0u, 0u, 0u};
      if (key < L) {
        // non-temporal: K / V rows are read once per (sequence, head) -- kept out of L2 for the
        // GEMM panels and the ctx rows the next projection reads (round 6: encode +0.4-0.8 % in three
        // alternating rounds, profiles/r06y/)
        kv[u] = __builtin_nontemporal_load((const u32x4*)(Kg + (int64_t)key * ld + c8 * 8));
        vv[u] = __builtin_nontemporal_load((const u32x4*)(Vg + (int64_t)key * ld + c8 * 8));
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int key = kp + kg * 4 + u;
      if (key < Lp) *(u32x4*)(Ks + key * 128 + ((c8 ^ ((key >> 1) & 7)) << 4)) = kv[u];
    }
    const int key0 = kp + kg * 4;
    if (key0 < Lp) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint16_t e[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) e[u] = ((const uint16_t*)&vv[u])[j];
        const uint32_t lo = (uint32_t)e[0] | ((uint32_t)e[1] << 16), hi = (uint32_t)e[2] | ((uint32_t)e[3] << 16);
        *(uint2*)(Vt + (c8 * 8 + j) * vts + key0 * 2) = make_uint2(lo, hi);
      }
    }
  }
  for (int i = tid; i < Lp; i += NT) {
    float bv = 0.0f;
    if (i >= L) bv = -3.402823466e+38f;
    else if (a.mask && a.mask[b * a.L + i] == 0) bv = -3.402823466e+38f;  // (1 - mask) * finfo.min
    kb[i] = bv;
  }
  __syncthreads();

  // per-lane LDS offsets (a 32-key tile starts at a multiple of 32 rows: its swizzle term never
  // depends on the tile)
  const int sw = (r >> 1) & 7;
  int offK[4];
#pragma unroll
  for (int st = 0; st < 4; ++st) offK[st] = r * 128 + ((((2 * st) | h) ^ sw) << 4);
  const int offV0 = r * vts + 8 * h, offV1 = (32 + r) * vts + 8 * h;
  const float inv = DROP ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const uint32_t thr = DROP ? attn_drop_threshold(a.drop_p) : 0u;
  bf16x8 oo[2][2];                           // NB: this wave's O block, [t][g / 2] (bf16)

  for (int qb = wave; qb < nqb; qb += NW) {
    // Q fragment (B operand, B[k=d][col=q] = Q[q][d]) scaled by 1/sqrt(dh)
    const int qq = qb * 32 + r;
    const int qrow = qq < L ? qq : L - 1;
    bf16x8 qf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 v = qb == wave ? q0[s] : *(const bf16x8*)(Qg + (int64_t)qrow * ld + s * 16 + h * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)((float)v[j] * a.scale);
      qf[s] = v;
    }
    const uint32_t rowkey = DROP ? attn_row_key(a.seed, a.site, (uint64_t)(hrow + qq)) : 0u;
    uint32_t words[NB ? NB : 1];               // keep words of this query (stored once, after the last tile)
    f32x16 o[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) o[t][e] = 0.0f;
    float m = -__builtin_inff(), l = 0.0f;

    auto tile = [&](int kt) {
      // S^T tile: rows = keys kt.., cols = queries
      f32x16 s;
#pragma unroll
      for (int e = 0; e < 16; ++e) s[e] = 0.0f;
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const bf16x8 kf = *(const bf16x8*)(Ks + kt * 128 + offK[st]);
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[st], s, 0, 0, 0);
      }
      // element pairs on the packed FP32 path (v_pk_fma_f32 / v_pk_add_f32: two elements per issue)
      float mt = -__builtin_inff();
      const f32x2 l2e = {kLog2e, kLog2e};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 kbv = *(const f32x4*)(kb + kt + 8 * g + 4 * h);
        const f32x2 lo = __builtin_elementwise_fma(f32x2{s[4 * g], s[4 * g + 1]}, l2e, f32x2{kbv[0], kbv[1]});
        const f32x2 hi = __builtin_elementwise_fma(f32x2{s[4 * g + 2], s[4 * g + 3]}, l2e, f32x2{kbv[2], kbv[3]});
        s[4 * g] = lo[0];
        s[4 * g + 1] = lo[1];
        s[4 * g + 2] = hi[0];
        s[4 * g + 3] = hi[1];
        mt = fmaxf(fmaxf(mt, fmaxf(s[4 * g], s[4 * g + 1])), fmaxf(s[4 * g + 2], s[4 * g + 3]));
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const bool grow = mt > m + kLazy;
      if (__builtin_amdgcn_ballot_w64(grow) != 0ull) {   // rare after the first tile
        const float mn = grow ? mt : m;
        const float alpha = __builtin_amdgcn_exp2f(m - mn);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int e = 0; e < 16; ++e) o[t][e] *= alpha;
        l *= alpha;
        m = mn;
      }
      const f32x2 mm = {m, m};
      f32x2 psum = {0.0f, 0.0f};
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        f32x2 v = f32x2{s[e], s[e + 1]} - mm;
        v[0] = __builtin_amdgcn_exp2f(v[0]);
        v[1] = __builtin_amdgcn_exp2f(v[1]);
        psum += v;
        s[e] = v[0];
        s[e + 1] = v[1];
      }
      float ps = psum[0] + psum[1];
      ps += __shfl_xor(ps, 32, 64);
      l += ps;
      if (DROP) {   // this lane's keys kt + 8 g + 4 h + {0,1,2,3}: pairs kt / 2 + 4 g + 2 h + {0, 1}
        const uint32_t pbase = rowkey + (uint32_t)((kt >> 1) + 2 * h) * kAttnPairStep;
        uint32_t m16 = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int u2 = 0; u2 < 2; ++u2) {
            const uint32_t hsh = attn_mix(pbase + (uint32_t)(4 * g + u2) * kAttnPairStep);
#pragma unroll
            for (int w = 0; w < 2; ++w) {
              const int e = 4 * g + 2 * u2 + w;
              const int kr = 8 * g + 4 * h + 2 * u2 + w;
              const bool keep = kt + kr < L && (w ? hsh >> 16 : hsh & 0xFFFFu) >= thr;
              m16 |= keep ? 1u << kr : 0u;
              s[e] = keep ? s[e] : 0.0f;
            }
          }
        if (a.drop_bits) {   // this query's 32 keep bits of the key tile: the two lane halves' 16 each
          const uint32_t word = m16 | __shfl_xor(m16, 32, 64);
          if (NB) words[NB ? (kt / 32) % NB : 0] = word;
          else if (h == 0 && qq < L) a.drop_bits[(hrow + qq) * nqb + kt / 32] = word;
        }
      }
      // O^T += V^T P^T over the 32 keys (2 k-steps of 16)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (__bf16)s[8 * ks + j];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const char* vrow = Vt + (t ? offV1 : offV0) + (kt + 16 * ks) * 2;
          const bf16x4 v0 = *(const bf16x4*)(vrow);
          const bf16x4 v1 = *(const bf16x4*)(vrow + 16);
          bf16x8 vf;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            vf[j] = v0[j];
            vf[4 + j] = v1[j];
          }
          o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[t], 0, 0, 0);
        }
      }
    };
    if (NB) {
#pragma unroll
      for (int j = 0; j < (NB ? NB : 1); ++j) tile(32 * j);
      if (DROP && a.drop_bits && h == 0 && qq < L) {   // the row's words: contiguous over the wave's queries
        uint32_t* dst = a.drop_bits + (hrow + qq) * nqb;
        if (NB == 4) {
          *(u32x4*)dst = u32x4{words[0], words[NB > 1 ? 1 : 0], words[NB > 2 ? 2 : 0], words[NB > 3 ? 3 : 0]};
        } else {
#pragma unroll
          for (int j = 0; j < (NB ? NB : 1); ++j) dst[j] = words[j];
        }
      }
    } else {
      for (int kt = 0; kt < Lp; kt += 32) tile(kt);
    }
    // O^T[d][q]: lane holds query r; d = 32t + (e&3) + 8(e>>2) + 4h
    if (qq < L && a.lse && h == 0) a.lse[hrow + qq] = (m + __log2f(l)) * kLn2;
    const float sc = inv / l;
    if (NB) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) oo[t][e >> 3][e & 7] = (__bf16)(o[t][e] * sc);
    } else if (qq < L) {
      __bf16* orow = a.ctx + (row0 + qq) * a.H + hd * kHeadDim;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 v;
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = (__bf16)(o[t][4 * g + u] * sc);
          *(bf16x4*)(orow + 32 * t + 8 * g + 4 * h) = v;
        }
    }
  }
  if (NB) {
    // O through LDS (the K image, dead once every wave is past its last tile): rows of 128 B
    __syncthreads();
    if (wave < nqb) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 v;
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = oo[t][g >> 1][(g & 1) * 4 + u];
          const int qr = wave * 32 + r, d0 = 32 * t + 8 * g + 4 * h;   // 4 consecutive d of row qr
          *(bf16x4*)(Ks + qr * 128 + (((d0 >> 3) ^ ((qr >> 1) & 7)) << 4) + (d0 & 7) * 2) = v;
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < (Lp * 8 + NT - 1) / NT; ++it) {
      const int i = tid + it * NT;
      const int row = i >> 3, c = i & 7;
      if (i < Lp * 8 && row < L)
        *(bf16x8*)(a.ctx + (row0 + row) * a.H + hd * kHeadDim + c * 8) =
            *(const bf16x8*)(Ks + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
    }
  }
}


// ---------------------------------------------------------------------------
// Pooling (utils.py:233-240, biencoder.py:139-146) and L2 normalisation.
// mode 0 = first ([CLS]), 1 = mean over mask, 2 = max of hidden*mask.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pool_kernel(const __bf16* hidden, const int64_t* mask, int64_t B, int64_t L,
                                                   int H, int mode, float* out, __bf16* out_bf16) {
  const int64_t b = blockIdx.x;
  for (int c = threadIdx.x; c < H; c += 256) {
    float v;
    if (mode == 0) {
      v = (float)hidden[(b * L) * H + c];
    } else if (mode == 1) {
      float s = 0.f, cnt = 0.f;
      for (int64_t l = 0; l < L; ++l) {
        const float mk = mask ? (float)mask[b * L + l] : 1.0f;
        s += (float)hidden[(b * L + l) * H + c] * mk;
        cnt += mk;
      }
      v = s / fmaxf(cnt, 1e-9f);
    } else {
      float mx = -__builtin_inff();
      for (int64_t l = 0; l < L; ++l) {
        const float mk = mask ? (float)mask[b * L + l] : 1.0f;
        mx = fmaxf(mx, (float)hidden[(b * L + l) * H + c] * mk);
      }
      v = mx;
    }
    out[b * H + c] = v;
    if (out_bf16) out_bf16[b * H + c] = (__bf16)v;
  }
}

__global__ __launch_bounds__(256) void l2norm_kernel(float* x, int64_t B, int H, __bf16* out_bf16) {
  __shared__ float red[4];
  const int64_t b = blockIdx.x;
  float s = 0.f;
  for (int c = threadIdx.x; c < H; c += 256) {
    const float v = x[b * H + c];
    s += v * v;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float den = fmaxf(sqrtf(tot), 1e-12f);  // F.normalize eps
  for (int c = threadIdx.x; c < H; c += 256) {
    const float v = x[b * H + c] / den;
    x[b * H + c] = v;
    if (out_bf16) out_bf16[b * H + c] = (__bf16)v;
  }
}

}  // namespace drt

using namespace drt;

extern "C" {

int drt_embed_ln_pre(const int64_t* ids, const int64_t* type_ids, int64_t B, int64_t L, const float* word_emb,
                     const float* pos_emb, const float* type_emb, const float* gamma, const float* beta, float eps,
                     int32_t H, void* out, void* pre, void* stream);

int drt_gelu_bf16(const void* x, int64_t n, void* y, void* stream) {
  DRT_REQUIRE(n >= 0);
  if (n == 0) return DRT_OK;
  DRT_REQUIRE(x && y);
  DRT_REQUIRE((uintptr_t)x % 16 == 0 && (uintptr_t)y % 16 == 0);
  hipLaunchKernelGGL(gelu_kernel, dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)x, n, (__bf16*)y);
  return hip_status(hipGetLastError());
}

int drt_embedding_bwd_types(const int64_t* ids, const int64_t* type_ids, int32_t ntypes, const void* d, int64_t B,
                            int64_t L, int32_t H, int64_t padding_idx, float* dword, float* dpos, float* dtype,
                            void* stream) {
  DRT_REQUIRE(B >= 0 && L > 0 && H > 0 && ntypes >= 1 && (type_ids == nullptr || ntypes <= kMaxTypes));
  if (B == 0) return DRT_OK;
  DRT_REQUIRE(ids && d && dword && dpos && dtype);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(embedding_bwd_word_kernel, dim3((unsigned)(B * L)), dim3(256), 0, s, ids, (const __bf16*)d,
                     (int)H, padding_idx, dword);
  const unsigned cy = (unsigned)((H + 255) / 256), cz = (unsigned)((B + kPosChunk - 1) / kPosChunk);
  hipLaunchKernelGGL(embedding_bwd_pos_kernel, dim3((unsigned)L, cy, cz), dim3(256), 0, s, (const __bf16*)d, B, L,
                     (int)H, dpos);
  if (!type_ids) {
    hipLaunchKernelGGL(embedding_bwd_type0_kernel, dim3(cy), dim3(256), 0, s, (const float*)dpos, L, (int)H, dtype);
  } else {
    const int64_t T = B * L;
    hipLaunchKernelGGL(embedding_bwd_type_kernel, dim3(cy, (unsigned)((T + kTypeChunk - 1) / kTypeChunk)), dim3(256),
                       0, s, type_ids, (const __bf16*)d, T, (int)H, (int)ntypes, dtype);
  }
  return hip_status(hipGetLastError());
}

int drt_embedding_bwd(const int64_t* ids, const int64_t* type_ids, const void* d, int64_t B, int64_t L, int32_t H,
                      int64_t padding_idx, float* dword, float* dpos, float* dtype, void* stream) {
  return drt_embedding_bwd_types(ids, type_ids, type_ids ? 2 : 1, d, B, L, H, padding_idx, dword, dpos, dtype, stream);
}

int drt_embed_ln(const int64_t* ids, const int64_t* type_ids, int64_t B, int64_t L, const float* word_emb,
                 const float* pos_emb, const float* type_emb, const float* gamma, const float* beta, float eps,
                 int32_t H, void* out, void* stream) {
  return drt_embed_ln_pre(ids, type_ids, B, L, word_emb, pos_emb, type_emb, gamma, beta, eps, H, out, nullptr, stream);
}

int drt_embed_ln_pre(const int64_t* ids, const int64_t* type_ids, int64_t B, int64_t L, const float* word_emb,
                     const float* pos_emb, const float* type_emb, const float* gamma, const float* beta, float eps,
                     int32_t H, void* out, void* pre, void* stream) {
  DRT_REQUIRE(B >= 0 && L > 0 && H > 0 && H % 256 == 0 && H <= 1024);
  const int64_t T = B * L;
  if (T == 0) return DRT_OK;
  DRT_REQUIRE(ids && word_emb && pos_emb && type_emb && gamma && beta && out);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((T + 3) / 4));
  __bf16* o = (__bf16*)out;
  __bf16* p = (__bf16*)pre;
#define EMB(E) hipLaunchKernelGGL(embed_ln_kernel<E>, grid, dim3(256), 0, s, ids, type_ids, T, L, word_emb, pos_emb, \
                                  type_emb, gamma, beta, eps, (int)H, o, p)
  switch (H / 64) {
    case 4: EMB(4); break;
    case 8: EMB(8); break;
    case 12: EMB(12); break;
    case 16: EMB(16); break;
    default: return DRT_EINVAL;
  }
#undef EMB
  return hip_status(hipGetLastError());
}

int drt_layernorm_f32_bf16(const float* X, int64_t M, int32_t H, const float* gamma, const float* beta, float eps,
                           void* out, void* stream) {
  DRT_REQUIRE(M >= 0 && H > 0 && H % 256 == 0 && H <= 1024);
  if (M == 0) return DRT_OK;
  DRT_REQUIRE(X && gamma && beta && out);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((M + 3) / 4));
  switch (H / 64) {
    case 4: hipLaunchKernelGGL(layernorm_f32_kernel<4>, grid, dim3(256), 0, s, X, M, H, gamma, beta, eps, (__bf16*)out); break;
    case 8: hipLaunchKernelGGL(layernorm_f32_kernel<8>, grid, dim3(256), 0, s, X, M, H, gamma, beta, eps, (__bf16*)out); break;
    case 12: hipLaunchKernelGGL(layernorm_f32_kernel<12>, grid, dim3(256), 0, s, X, M, H, gamma, beta, eps, (__bf16*)out); break;
    case 16: hipLaunchKernelGGL(layernorm_f32_kernel<16>, grid, dim3(256), 0, s, X, M, H, gamma, beta, eps, (__bf16*)out); break;
    default: return DRT_EINVAL;
  }
  return hip_status(hipGetLastError());
}

int drt_layernorm_bf16(const void* X, int64_t M, int32_t H, const float* gamma, const float* beta, float eps,
                       void* out, void* stream) {
  DRT_REQUIRE(M >= 0 && H > 0 && H % 256 == 0 && H <= 1024);
  if (M == 0) return DRT_OK;
  DRT_REQUIRE(X && gamma && beta && out);
  hipStream_t s = (hipStream_t)stream;
  const __bf16* x = (const __bf16*)X;
  __bf16* o = (__bf16*)out;
  dim3 grid(ln_rows_grid(M));
  switch (H / 64) {
    case 4: hipLaunchKernelGGL(layernorm_bf16_kernel<4>, grid, dim3(256), 0, s, x, M, H, gamma, beta, eps, o); break;
    case 8: hipLaunchKernelGGL(layernorm_bf16_kernel<8>, grid, dim3(256), 0, s, x, M, H, gamma, beta, eps, o); break;
    case 12: hipLaunchKernelGGL(layernorm_bf16_kernel<12>, grid, dim3(256), 0, s, x, M, H, gamma, beta, eps, o); break;
    case 16: hipLaunchKernelGGL(layernorm_bf16_kernel<16>, grid, dim3(256), 0, s, x, M, H, gamma, beta, eps, o); break;
    default: return DRT_EINVAL;
  }
  return hip_status(hipGetLastError());
}

int drt_attention_fwd_lse_bf16(const void* qkv, const int64_t* mask, void* ctx, float* lse, int64_t B, int64_t L,
                               int32_t heads, int32_t head_dim, float scale, void* stream);

int drt_attention_bf16(const void* qkv, const int64_t* mask, void* ctx, int64_t B, int64_t L, int32_t heads,
                       int32_t head_dim, float scale, void* stream) {
  return drt_attention_fwd_lse_bf16(qkv, mask, ctx, nullptr, B, L, heads, head_dim, scale, stream);
}

int drt_attention_train_fwd_bf16(const void* qkv, const int64_t* mask, void* ctx, float* lse, int64_t B, int64_t L,
                                 int32_t heads, int32_t head_dim, float scale, float drop_p, uint64_t seed,
                                 uint64_t site, void* stream);

int drt_attention_fwd_lse_bf16(const void* qkv, const int64_t* mask, void* ctx, float* lse, int64_t B, int64_t L,
                               int32_t heads, int32_t head_dim, float scale, void* stream) {
  return drt_attention_train_fwd_bf16(qkv, mask, ctx, lse, B, L, heads, head_dim, scale, 0.0f, 0, 0, stream);
}

int drt_attention_train_fwd_bits_bf16(const void* qkv, const int64_t* mask, void* ctx, float* lse,
                                      uint32_t* drop_bits, int64_t B, int64_t L, int32_t heads, int32_t head_dim,
                                      float scale, float drop_p, uint64_t seed, uint64_t site, void* stream);

int drt_attention_train_fwd_bf16(const void* qkv, const int64_t* mask, void* ctx, float* lse, int64_t B, int64_t L,
                                 int32_t heads, int32_t head_dim, float scale, float drop_p, uint64_t seed,
                                 uint64_t site, void* stream) {
  return drt_attention_train_fwd_bits_bf16(qkv, mask, ctx, lse, nullptr, B, L, heads, head_dim, scale, drop_p, seed,
                                           site, stream);
}

// The training forward that also writes the attention-dropout keep mask as bits (drop_bits, when
// drop_p > 0 and drop_bits != NULL): [B][heads][L][ceil(L / 32)] u32, bit (key & 31) of word
// (query, key >> 5); drt_attention_train_bwd_bits_bf16 reads it instead of regenerating the hash.
int drt_attention_train_fwd_bits_bf16(const void* qkv, const int64_t* mask, void* ctx, float* lse,
                                      uint32_t* drop_bits, int64_t B, int64_t L, int32_t heads, int32_t head_dim,
                                      float scale, float drop_p, uint64_t seed, uint64_t site, void* stream) {
  DRT_REQUIRE(B >= 0 && L > 0 && L <= kMaxSeq && heads > 0 && head_dim == kHeadDim);
  DRT_REQUIRE(drop_p >= 0.0f && drop_p < 1.0f);
  if (B == 0) return DRT_OK;
  DRT_REQUIRE(qkv && ctx);
  AttnArgs a{(const __bf16*)qkv, mask, (__bf16*)ctx, B, L, heads, heads * head_dim, scale, lse, drop_p, seed, site,
             drop_bits};
  const int Lp = ((int)L + 31) & ~31;
  const int nb = Lp / 32;
  const size_t lds = (size_t)Lp * 128 + (size_t)64 * (Lp * 2 + 8) + (size_t)Lp * 4;
  static bool attr_set = false;
  if (!attr_set) {
    const void* ks[] = {(const void*)attention_fwd_kernel<0, false>, (const void*)attention_fwd_kernel<4, false>,
                        (const void*)attention_fwd_kernel<5, false>, (const void*)attention_fwd_kernel<4, true>,
                        (const void*)attention_fwd_kernel<5, true>, (const void*)attention_fwd_kernel<0, true>};
    for (const void* f : ks) DRT_CHECK_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  const dim3 grid((unsigned)(B * heads));
  hipStream_t s = (hipStream_t)stream;
  const bool drop = drop_p > 0.0f;
#define DRT_AF_LAUNCH(NB_)                                                                              \
  case NB_: {                                                                                           \
    const dim3 blk(NB_ == 5 ? 320 : 256);                                                               \
    if (drop) hipLaunchKernelGGL((attention_fwd_kernel<NB_, true>), grid, blk, lds, s, a);             \
    else hipLaunchKernelGGL((attention_fwd_kernel<NB_, false>), grid, blk, lds, s, a);                 \
    break;                                                                                              \
  }
  switch (nb) {
    DRT_AF_LAUNCH(1)
    DRT_AF_LAUNCH(2)
    DRT_AF_LAUNCH(3)
    DRT_AF_LAUNCH(4)
    DRT_AF_LAUNCH(5)
    default:   // 161 <= L <= 512 (the backward's streamed kernels)
      if (drop) hipLaunchKernelGGL((attention_fwd_kernel<0, true>), grid, dim3(256), lds, s, a);
      else hipLaunchKernelGGL((attention_fwd_kernel<0, false>), grid, dim3(256), lds, s, a);
      break;
  }
#undef DRT_AF_LAUNCH
  return hip_status(hipGetLastError());
}

int drt_pool_bf16(const void* hidden, const int64_t* mask, int64_t B, int64_t L, int32_t H, int32_t mode,
                  float* out, void* out_bf16, void* stream) {
  DRT_REQUIRE(B >= 0 && L > 0 && H > 0 && mode >= 0 && mode <= 2);
  if (B == 0) return DRT_OK;
  DRT_REQUIRE(hidden && out);
  hipLaunchKernelGGL(pool_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, (const __bf16*)hidden, mask,
                     B, L, H, mode, out, (__bf16*)out_bf16);
  return hip_status(hipGetLastError());
}

int drt_l2_normalize_f32(float* x, int64_t B, int32_t H, void* out_bf16, void* stream) {
  DRT_REQUIRE(B >= 0 && H > 0);
  if (B == 0) return DRT_OK;
  DRT_REQUIRE(x);
  hipLaunchKernelGGL(l2norm_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, x, B, H, (__bf16*)out_bf16);
  return hip_status(hipGetLastError());
}

}  // extern "C"
