// match.hip -- answer matching of retrieved passages (has_answers, DRT/evaluator/nq_eval.py:187-218)
// on token ids already in HBM (evaluator/nq_eval.py DeviceRowMatcher).
//
// The reference re-tokenises each of a query's k retrieved passages and scans it for every answer's
// token sequence on the host.  Here every passage of the index has its uncased token ids in one
// padded [slots, W] int32 matrix resident on the GPU (tokenised once per evaluation on the host,
// -1 pads) with the row -> slot table beside it; a query batch is ONE launch: wave (i, j) takes
// retrieved row j of query i (its slot looked up on the device), its lanes take
// window starts s, and the row matches when some answer a of query i has tok[s + t] == ans[a][t]
// for every t < len(a) (s + len(a) <= W).  Unknown answer tokens (id -2 on the host) never equal a
// passage token; an empty answer -- `every` -- matches every passage, as the reference's loop does.
#include "drt_common.h"

namespace drt {

constexpr int kMatchWaves = 4;

__global__ __launch_bounds__(kMatchWaves * 64) void answer_match_kernel(const int32_t* tok, int W,
                                                                        const int64_t* rows, const int64_t* slot_of,
                                                                        int64_t n_rows, int64_t B, int64_t k,
                                                                        const int32_t* ans, const int32_t* alen, int A,
                                                                        int n_max, const uint8_t* every, int8_t* hit) {
  const int lane = threadIdx.x & 63;
  const int64_t pair = (int64_t)blockIdx.x * kMatchWaves + (threadIdx.x >> 6);   // i * k + j
  if (pair >= B * k) return;
  const int64_t i = pair / k;
  const int64_t row = rows[pair];
  const int64_t slot = slot_of ? ((row >= 0 && row < n_rows) ? slot_of[row] : -1) : row;
  if (slot < 0) {   // pad row (id -1) or a row without tokens: never a hit
    if (lane == 0) hit[pair] = 0;
    return;
  }
  if (every[i]) {
    if (lane == 0) hit[pair] = 1;
    return;
  }
  const int32_t* trow = tok + slot * (int64_t)W;
  const int32_t* qa = ans + i * (int64_t)A * n_max;
  const int32_t* ql = alen + i * (int64_t)A;
  bool found = false;
  for (int s = lane; s < W && !found; s += 64) {
    for (int a = 0; a < A && !found; ++a) {
      const int n = ql[a];
      if (n <= 0 || s + n > W) continue;
      bool m = true;
      for (int t = 0; t < n && m; ++t) m = trow[s + t] == qa[a * n_max + t];
      found = m;
    }
  }
  const bool any = __ballot(found) != 0ull;
  if (lane == 0) hit[pair] = any ? 1 : 0;
}

}  // namespace drt

using namespace drt;

extern "C" {

int drt_answer_match_i32(const int32_t* tok, int32_t W, const int64_t* rows, const int64_t* slot_of, int64_t n_rows,
                         int64_t B, int64_t k, const int32_t* ans, const int32_t* alen, int32_t A, int32_t n_max,
                         const uint8_t* every, int8_t* hit, void* stream) {
  DRT_REQUIRE(B >= 0 && k >= 0 && W > 0 && A >= 1 && n_max >= 1 && n_rows >= 0);
  if (B == 0 || k == 0) return DRT_OK;
  DRT_REQUIRE(tok && rows && ans && alen && every && hit);
  const int64_t pairs = B * k;
  hipLaunchKernelGGL(answer_match_kernel, dim3((unsigned)((pairs + kMatchWaves - 1) / kMatchWaves)),
                     dim3(kMatchWaves * 64), 0, (hipStream_t)stream, tok, (int)W, rows, slot_of, n_rows, B, k, ans,
                     alen, (int)A, (int)n_max, every, hit);
  return hip_status(hipGetLastError());
}

}  // extern "C"
