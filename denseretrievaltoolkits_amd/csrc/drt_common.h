// Shared device/host helpers for the DRT MI355X (gfx950) kernels.
//
// Everything here is CDNA4-only: 64-lane waves, MFMA bf16 tiles, LDS-DMA
// (global_load_lds) staging.  No CUDA shims, no dual paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/drt.h"

namespace drt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));   // v_pk_{fma,mul,add}_f32 operand pair
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(3))) void lds_void;

// ---------------------------------------------------------------------------
// Order-preserving key for (score desc, row asc).
//
// faiss IndexFlatIP returns hits by descending inner product
// (DRT/evaluator/index.py:31-33 re-sorts them with np.argsort(-scores)); the
// reference leaves the order of equal scores unspecified, the build pins it to
// ascending row/doc id.  `desc_key(s)` is a uint32 whose ASCENDING order is the
// DESCENDING order of s; (desc_key << 32 | row) then sorts ascending exactly in
// (score desc, row asc) order.  -0.0 is folded onto +0.0 first (numpy treats
// them as equal).
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t desc_key(float s) {
  s = s + 0.0f;
  uint32_t u = __builtin_bit_cast(uint32_t, s);
  uint32_t ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // ascending order
  return ~ord;                                                 // descending order
}

__host__ __device__ __forceinline__ float desc_key_to_score(uint32_t k) {
  uint32_t ord = ~k;
  uint32_t u = (ord & 0x80000000u) ? (ord & 0x7FFFFFFFu) : ~ord;
  return __builtin_bit_cast(float, u);
}

// Score histograms of the select / threshold kernels.  hist_scale: bins per unit score, 0 when the
// range is degenerate (empty, subnormal-small so that nbins / range overflows, infinite or NaN) --
// every key then falls in one bin and the callers' exact fallbacks take over.  hist_bin: the bin
// of f = distance * scale, clamped to [0, nbins) without an out-of-range or NaN float -> int
// conversion; a NaN distance (a NaN score) goes to `nan_bin`, the end of the histogram its key
// sorts to (desc_key: a positive NaN above +inf, a negative one below -inf).
__device__ __forceinline__ float hist_scale(float nbins, float range) {
  const float s = nbins / range;
  return (range > 0.0f && __builtin_isfinite(s)) ? s : 0.0f;
}
__device__ __forceinline__ int hist_bin(float f, int nbins, int nan_bin) {
  if (f != f) return nan_bin;
  if (!(f < (float)(nbins - 1))) return nbins - 1;
  return f < 1.0f ? 0 : (int)f;
}

// Training dropout (HF BertModel in train mode: embeddings, attention probabilities, and the
// two sublayer outputs, modeling_bert.py:107,195,296,348): a counter-based hash of (seed, site,
// element index) decides each keep, so forward and backward regenerate the same mask without
// storing it; keep iff the top 24 hash bits >= p * 2^24.  model/train_tower.py restates it in
// torch for the tests.
__host__ __device__ __forceinline__ uint32_t drop_hash24(uint64_t seed, uint64_t site, uint64_t idx) {
  uint64_t x = idx * 0x9E3779B97F4A7C15ull + seed + site * 0xBF58476D1CE4E5B9ull;
  x ^= x >> 31;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 29;
  return (uint32_t)(x >> 40);
}
__host__ __device__ __forceinline__ uint32_t drop_threshold(float p) { return (uint32_t)(p * 16777216.0f); }

// Attention-probability dropout (modeling_bert.py:195) is the one site with L x L decisions per
// (sequence, head), so it draws two per hash and keeps the 64-bit arithmetic out of the per-element
// path: row = (b * heads + head) * L + query gets a 32-bit row key from the 64-bit mixer above (once
// per query row); key pair j = key >> 1 hashes to fmix32(row_key + j * 0x9E3779B9) (murmur3's
// finaliser on a Weyl sequence: two 32-bit multiplies per pair); the low 16 bits decide the even key,
// the high 16 the odd one; keep iff half >= p * 2^16.
constexpr uint32_t kAttnPairStep = 0x9E3779B9u;
__host__ __device__ __forceinline__ uint32_t attn_row_key(uint64_t seed, uint64_t site, uint64_t row) {
  uint64_t x = row * 0x9E3779B97F4A7C15ull + seed + site * 0xBF58476D1CE4E5B9ull;
  x ^= x >> 31;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 29;
  return (uint32_t)(x >> 32);
}
__host__ __device__ __forceinline__ uint32_t attn_mix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__host__ __device__ __forceinline__ uint32_t attn_drop_threshold(float p) { return (uint32_t)(p * 65536.0f); }
// keep decision of (row key, key) -- the per-element form of the pairwise draw
__host__ __device__ __forceinline__ bool attn_keep(uint32_t row_key, int key, uint32_t thr16) {
  const uint32_t hsh = attn_mix(row_key + (uint32_t)(key >> 1) * kAttnPairStep);
  return ((key & 1) ? hsh >> 16 : hsh & 0xFFFFu) >= thr16;
}

constexpr float kLog2e = 1.4426950408889634f;   // softmax in exp2 form (attention kernels)

// faiss pads rows that have fewer than k results with label -1 and the
// lowest float (CMin<float>::neutral() == numeric_limits<float>::lowest()).
constexpr float kPadScore = -3.402823466e+38f;

inline int hip_status(hipError_t e) { return e == hipSuccess ? DRT_OK : (int)e; }

#define DRT_CHECK_HIP(expr)                  \
  do {                                       \
    hipError_t _e = (expr);                  \
    if (_e != hipSuccess) return (int)_e;    \
  } while (0)

#define DRT_REQUIRE(cond)                    \
  do {                                       \
    if (!(cond)) return DRT_EINVAL;          \
  } while (0)

}  // namespace drt
