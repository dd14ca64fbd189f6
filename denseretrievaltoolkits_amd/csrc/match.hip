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

// get_metrics (DRT/evaluator/metrics.py:4-59) of one loader batch's hit matrix hit [B][k], added to the
// evaluation's running sums on the device (Trainer.evaluate reads them back once): for each cut-off k_t,
//   acc[t]         += recall@k_t = #rows whose first hit is at position < k_t,
//   acc[T + t]     += mrr@k_t    = sum over those rows of 1 / (first + 1),
//   acc[2 T + t]   += ndcg@k_t   = sum_rows DCG@k_t / sum_rows IDCG@k_t (a batch-level ratio; natural-log
//                   discounts 1 / ln(j + 2); IDCG over max(#hits in the row, 1) ideal positions).
// One 1024-thread work-group: column hit counts and per-row first hit / count in parallel, then the
// prefix sums and the per-cut-off totals in the order metrics.py's numpy takes them (cumsum).
constexpr int kMetricThreads = 1024;
constexpr int kMetricMaxK = 2048;
constexpr int kMetricMaxB = 4096;
constexpr int kMetricMaxT = 16;

__global__ __launch_bounds__(kMetricThreads) void hit_metrics_kernel(const int8_t* hit, int64_t B, int64_t k,
                                                                     const int32_t* topk, int T, double* acc) {
  __shared__ double disc[kMetricMaxK];
  __shared__ double cumdisc[kMetricMaxK + 1];
  __shared__ double cumdcg[kMetricMaxK + 1];
  __shared__ int ccount[kMetricMaxK];
  __shared__ int first[kMetricMaxB];
  __shared__ int cnt[kMetricMaxB];
  for (int64_t j = threadIdx.x; j < k; j += kMetricThreads) {
    disc[j] = 1.0 / log((double)(j + 2));
    int c = 0;
    for (int64_t b = 0; b < B; ++b) c += hit[b * k + j] != 0 ? 1 : 0;
    ccount[j] = c;
  }
  for (int64_t b = threadIdx.x; b < B; b += kMetricThreads) {
    const int8_t* hr = hit + b * k;
    int f = -1, c = 0;
    for (int64_t j = 0; j < k; ++j) {
      const bool h = hr[j] != 0;
      if (h && f < 0) f = (int)j;
      c += h ? 1 : 0;
    }
    first[b] = f;
    cnt[b] = c;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  cumdisc[0] = 0.0;
  cumdcg[0] = 0.0;
  for (int64_t j = 0; j < k; ++j) {   // numpy's cumsum order
    cumdisc[j + 1] = cumdisc[j] + disc[j];
    cumdcg[j + 1] = cumdcg[j] + (double)ccount[j] * disc[j];
  }
  for (int t = 0; t < T; ++t) {
    const int64_t kt = topk[t];
    int64_t rec = 0;
    double mrr = 0.0, idcg = 0.0, dcg = 0.0;
    for (int64_t b = 0; b < B; ++b) {
      if (first[b] >= 0 && first[b] < kt) {
        ++rec;
        mrr += 1.0 / (double)(first[b] + 1);
      }
      int64_t n = cnt[b] > 1 ? cnt[b] : 1;   // ideal positions: max(#hits, 1), at most k_t (and k)
      n = n < kt ? n : kt;
      n = n < k ? n : k;
      idcg += cumdisc[n];
    }
    const int64_t kk = kt < k ? kt : k;
    dcg = cumdcg[kk];
    acc[t] += (double)rec;
    acc[T + t] += mrr;
    acc[2 * T + t] += idcg != 0.0 ? dcg / idcg : __builtin_nan("");
  }
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

int drt_hit_metrics_i8(const int8_t* hit, int64_t B, int64_t k, const int32_t* topk, int32_t T, double* acc,
                       void* stream) {
  DRT_REQUIRE(B >= 0 && k >= 0 && k <= kMetricMaxK && B <= kMetricMaxB && T >= 1 && T <= kMetricMaxT);
  if (B == 0) return DRT_OK;
  DRT_REQUIRE(hit && topk && acc);
  hipLaunchKernelGGL(hit_metrics_kernel, dim3(1), dim3(kMetricThreads), 0, (hipStream_t)stream, hit, B, k, topk,
                     (int)T, acc);
  return hip_status(hipGetLastError());
}

}  // extern "C"
