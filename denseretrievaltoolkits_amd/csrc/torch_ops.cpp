// torch_ops.cpp — PyTorch-ROCm custom operators (torch.ops.drt.*) over the C ABI of drt.h.
//
// Thin host-side adapters: shape/dtype checks (TORCH_CHECK -> Python RuntimeError), output and
// workspace tensors from torch's caching allocator, work enqueued on the current HIP stream of
// the inputs' device, then one call into libdrt_hip.so.  No arithmetic lives here.
//
// Reference sites these ops stand in for (see include/drt.h for the per-function mapping):
//   faiss.IndexFlatIP.search           DRT/evaluator/index.py:31-33        drt::ip_topk(+_resolve)
//   per-partition merge                DRT/model/utils.py:215-229          drt::topk_merge, merge_packed
//   corpus sharding (file exchange)    DRT/trainer/trainer.py:191-262      drt::dist_sample/_tau/_filter
//   score matrix + CE (+ autograd)     DRT/model/biencoder.py:107-119      drt::score_ce_fwd/_bwd
//   HF BertModel forward pieces        transformers modeling_bert.py       drt::embed_ln, linear,
//                                                                          attention, layernorm, pool,
//                                                                          l2_normalize
// Fake (meta) kernels and the autograd formula of score_ce_fwd are registered from Python
// (denseretrievaltoolkits_amd/ops.py).
#include <vector>

#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
// torch-ROCm exposes GPU tensors under the "cuda" device type; its HIP streams are reached
// through the MasqueradingAsCUDA view of c10_hip (the HIP stream itself, no CUDA API)
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "drt.h"

namespace {

using at::Tensor;

void* stream_of(const Tensor& t) {
  return (void*)at::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

// argument errors surface as Python ValueError (TORCH_CHECK_VALUE), HIP failures as RuntimeError
void check_rc(int rc, const char* what) {
  TORCH_CHECK_VALUE(rc != DRT_EINVAL, what, ": invalid argument (DRT_EINVAL)");
  TORCH_CHECK(rc == DRT_OK, what, ": HIP error ", rc);
}

void need_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "drt ops run on the GPU only (", name, " is on ", t.device(),
              "; no CPU fallback exists)");
}

void need(const Tensor& t, const char* name, at::ScalarType dt, int64_t dim) {
  need_gpu(t, name);
  TORCH_CHECK_VALUE(t.scalar_type() == dt, name, ": expected ", dt, ", got ", t.scalar_type());
  TORCH_CHECK_VALUE(t.dim() == dim, name, ": expected a ", dim, "-d tensor, got ", t.dim(), "-d");
}

const void* ptr_or_null(const c10::optional<Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

Tensor workspace(const Tensor& like, size_t bytes) {
  return at::empty({(int64_t)std::max<size_t>(bytes, 1)}, like.options().dtype(at::kByte));
}

// ---------------------------------------------------------------------------- search
// The caller-provided result buffers of ip_topk.out / ip_topk_resolve: the kernels write through their
// raw pointers, so shape, dtype, contiguity and device are checked before any launch.
static void check_topk_outputs(const Tensor& q, int64_t nq, int64_t k, const Tensor& scores, const Tensor& ids,
                               const Tensor& status) {
  TORCH_CHECK_VALUE(scores.device() == q.device() && ids.device() == q.device() && status.device() == q.device(),
                    "scores / ids / status must be on the queries' device ", q.device());
  TORCH_CHECK_VALUE(scores.is_contiguous() && scores.scalar_type() == at::kFloat && scores.dim() == 2 &&
                        scores.size(0) == nq && scores.size(1) == k,
                    "scores: expected a contiguous float [", nq, ", ", k, "] tensor, got ", scores.sizes());
  TORCH_CHECK_VALUE(ids.is_contiguous() && ids.scalar_type() == at::kLong && ids.dim() == 2 && ids.size(0) == nq &&
                        ids.size(1) == k,
                    "ids: expected a contiguous int64 [", nq, ", ", k, "] tensor, got ", ids.sizes());
  TORCH_CHECK_VALUE(status.is_contiguous() && status.scalar_type() == at::kInt && status.dim() == 1 &&
                        status.size(0) == nq,
                    "status: expected a contiguous int32 [", nq, "] tensor, got ", status.sizes());
}

// row statistics of the canonical-order stage: a [DRT_ROW_STATS_LEN] float tensor on p's device
// (drt_row_stats_bf16)
static const float* stats_ptr(const c10::optional<Tensor>& stats, const Tensor& q) {
  if (!stats.has_value()) return nullptr;
  TORCH_CHECK_VALUE(stats->device() == q.device() && stats->scalar_type() == at::kFloat &&
                        stats->numel() == DRT_ROW_STATS_LEN && stats->is_contiguous(),
                    "stats: expected a contiguous float [", DRT_ROW_STATS_LEN, "] tensor on ", q.device());
  return stats->data_ptr<float>();
}

void ip_topk_out(const Tensor& q_, const Tensor& p_, int64_t k, int64_t id_offset, const c10::optional<Tensor>& stats,
                 Tensor& scores, Tensor& ids, Tensor& status) {
  need(q_, "q", at::kBFloat16, 2);
  need(p_, "p", at::kBFloat16, 2);
  TORCH_CHECK_VALUE(q_.size(1) == p_.size(1), "q and p differ in dimension: ", q_.sizes(), " vs ", p_.sizes());
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous();
  const int64_t nq = q.size(0), n = p.size(0), d = q.size(1);
  check_topk_outputs(q, nq, k, scores, ids, status);
  const size_t wsb = drt_ip_topk_workspace(nq, n, (int32_t)d, (int32_t)k);
  TORCH_CHECK_VALUE(wsb > 0 || nq == 0, "unsupported ip_topk shape nq=", nq, " n=", n, " d=", d, " k=", k,
              " (d % 64 == 0, d <= 1024, 1 <= k <= 2048)");
  Tensor ws = workspace(q, wsb);
  const float* sp = stats_ptr(stats, q);
  if (sp) {
    check_rc(drt_ip_topk_exact_bf16(q.data_ptr(), nq, n ? p.data_ptr() : nullptr, n, (int32_t)d, (int32_t)k,
                                    id_offset, sp, scores.data_ptr<float>(), ids.data_ptr<int64_t>(),
                                    status.data_ptr<int32_t>(), ws.data_ptr(), wsb, stream_of(q)),
             "drt_ip_topk_exact_bf16");
  } else {
    check_rc(drt_ip_topk_bf16(q.data_ptr(), nq, n ? p.data_ptr() : nullptr, n, (int32_t)d, (int32_t)k, id_offset,
                              scores.data_ptr<float>(), ids.data_ptr<int64_t>(), status.data_ptr<int32_t>(),
                              ws.data_ptr(), wsb, stream_of(q)),
             "drt_ip_topk_bf16");
  }
}

std::tuple<Tensor, Tensor, Tensor> ip_topk(const Tensor& q, const Tensor& p, int64_t k, int64_t id_offset,
                                           const c10::optional<Tensor>& stats) {
  need_gpu(q, "q");
  const int64_t nq = q.size(0);
  Tensor s = at::empty({nq, k}, q.options().dtype(at::kFloat));
  Tensor i = at::empty({nq, k}, q.options().dtype(at::kLong));
  Tensor st = at::empty({nq}, q.options().dtype(at::kInt));
  ip_topk_out(q, p, k, id_offset, stats, s, i, st);
  return {s, i, st};
}

int64_t ip_topk_resolve(const Tensor& q_, const Tensor& p_, int64_t k, int64_t id_offset, Tensor& scores,
                        Tensor& ids, Tensor& status, const c10::optional<Tensor>& stats) {
  need(q_, "q", at::kBFloat16, 2);
  need(p_, "p", at::kBFloat16, 2);
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous();
  TORCH_CHECK_VALUE(q.size(1) == p.size(1), "q and p differ in dimension: ", q.sizes(), " vs ", p.sizes());
  TORCH_CHECK_VALUE(p.device() == q.device(), "q and p must be on the same device");
  const int64_t nq = q.size(0), n = p.size(0), d = q.size(1);
  TORCH_CHECK_VALUE(k >= 1 && k <= 2048, "unsupported k=", k);
  check_topk_outputs(q, nq, k, scores, ids, status);
  if (nq == 0) return 0;
  // bit 0 = not certified (bit 1, order not certified, cannot be improved by a rescan)
  const int64_t nbad = status.bitwise_and(1).ne(0).sum().item<int64_t>();   // synchronises, like the C entry
  if (nbad == 0) return 0;
  const size_t wsb = drt_ip_topk_resolve_workspace(nbad, n, (int32_t)d);
  Tensor ws = workspace(q, wsb);
  int64_t nres = 0;
  const float* sp = stats_ptr(stats, q);
  if (sp) {
    check_rc(drt_ip_topk_resolve_exact(q.data_ptr(), nq, n ? p.data_ptr() : nullptr, n, (int32_t)d, (int32_t)k,
                                       id_offset, sp, scores.data_ptr<float>(), ids.data_ptr<int64_t>(),
                                       status.data_ptr<int32_t>(), ws.data_ptr(), wsb, &nres, stream_of(q)),
             "drt_ip_topk_resolve_exact");
  } else {
    check_rc(drt_ip_topk_resolve(q.data_ptr(), nq, n ? p.data_ptr() : nullptr, n, (int32_t)d, (int32_t)k,
                                 id_offset, scores.data_ptr<float>(), ids.data_ptr<int64_t>(),
                                 status.data_ptr<int32_t>(), ws.data_ptr(), wsb, &nres, stream_of(q)),
             "drt_ip_topk_resolve");
  }
  return nres;
}

// canonical order of the queries whose status is exactly 2 (drt_ip_topk_resolve_wide): a filter pass at
// the lowered threshold, exact sums of what it collects, exact-key top-k in place; returns the number of
// queries whose bit 1 it cleared (synchronises, like the C entry)
int64_t ip_topk_resolve_wide(const Tensor& q_, const Tensor& p_, int64_t k, int64_t id_offset, Tensor& scores,
                             Tensor& ids, Tensor& status, const Tensor& stats) {
  need(q_, "q", at::kBFloat16, 2);
  need(p_, "p", at::kBFloat16, 2);
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous();
  TORCH_CHECK_VALUE(q.size(1) == p.size(1), "q and p differ in dimension: ", q.sizes(), " vs ", p.sizes());
  TORCH_CHECK_VALUE(p.device() == q.device(), "q and p must be on the same device");
  const int64_t nq = q.size(0), n = p.size(0), d = q.size(1);
  TORCH_CHECK_VALUE(k >= 1 && k <= 2048, "unsupported k=", k);
  check_topk_outputs(q, nq, k, scores, ids, status);
  const float* sp = stats_ptr(stats, q);
  if (nq == 0 || n == 0) return 0;
  const size_t wsb = drt_ip_topk_resolve_wide_workspace(n, (int32_t)d);
  TORCH_CHECK_VALUE(wsb > 0, "unsupported resolve_wide shape n=", n, " d=", d);
  Tensor ws = workspace(q, wsb);
  int64_t nres = 0;
  check_rc(drt_ip_topk_resolve_wide(q.data_ptr(), nq, p.data_ptr(), n, (int32_t)d, (int32_t)k, id_offset, sp,
                                    scores.data_ptr<float>(), ids.data_ptr<int64_t>(), status.data_ptr<int32_t>(),
                                    ws.data_ptr(), wsb, &nres, stream_of(q)),
           "drt_ip_topk_resolve_wide");
  return nres;
}

// top-k for 2048 < k <= 32768 in the canonical order (drt_ip_topk_large): tau [nq] = a lower bound of each
// query's k-th fp32 score; asynchronous, status 2 marks a query whose collected set overflowed
static std::tuple<Tensor, Tensor, Tensor, Tensor> ip_topk_large_impl(const Tensor& q_, const Tensor& p_, int64_t k,
                                                                     int64_t id_offset, const Tensor& stats,
                                                                     const Tensor& tau, bool want_keys) {
  need(q_, "q", at::kBFloat16, 2);
  need(p_, "p", at::kBFloat16, 2);
  need(tau, "tau", at::kFloat, 1);
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous();
  TORCH_CHECK_VALUE(q.size(1) == p.size(1), "q and p differ in dimension: ", q.sizes(), " vs ", p.sizes());
  TORCH_CHECK_VALUE(p.device() == q.device() && tau.device() == q.device(), "q, p and tau must share a device");
  const int64_t nq = q.size(0), n = p.size(0), d = q.size(1);
  TORCH_CHECK_VALUE(tau.size(0) == nq && tau.is_contiguous(), "tau must be a contiguous [nq] tensor");
  const size_t wsb = drt_ip_topk_large_workspace((int32_t)d, (int32_t)k);
  TORCH_CHECK_VALUE(wsb > 0, "unsupported ip_topk_large shape d=", d, " k=", k, " (d % 64 == 0, d <= 1024, k <= 32768)");
  const float* sp = stats_ptr(stats, q);
  Tensor scores = at::empty({nq, k}, q.options().dtype(at::kFloat));
  Tensor ids = at::empty({nq, k}, q.options().dtype(at::kLong));
  Tensor status = at::empty({nq}, q.options().dtype(at::kInt));
  Tensor keys = at::empty({want_keys ? nq : 0, k}, q.options().dtype(at::kLong));
  if (nq == 0) return {scores, ids, status, keys};
  Tensor ws = workspace(q, wsb);
  check_rc(drt_ip_topk_large_keys(q.data_ptr(), nq, n ? p.data_ptr() : nullptr, n, (int32_t)d, (int32_t)k, id_offset,
                                  sp, tau.data_ptr<float>(), scores.data_ptr<float>(), ids.data_ptr<int64_t>(),
                                  want_keys ? (uint64_t*)keys.data_ptr<int64_t>() : nullptr,
                                  status.data_ptr<int32_t>(), ws.data_ptr(), wsb, stream_of(q)),
           "drt_ip_topk_large_keys");
  return {scores, ids, status, keys};
}

std::tuple<Tensor, Tensor, Tensor> ip_topk_large(const Tensor& q, const Tensor& p, int64_t k, int64_t id_offset,
                                                 const Tensor& stats, const Tensor& tau) {
  auto r = ip_topk_large_impl(q, p, k, id_offset, stats, tau, false);
  return {std::get<0>(r), std::get<1>(r), std::get<2>(r)};
}

// the same plus each entry's exact order key (u64 bits in int64; ~0 = pad): the per-shard step of a
// sharded search at k > 2048
std::tuple<Tensor, Tensor, Tensor, Tensor> ip_topk_large_keys(const Tensor& q, const Tensor& p, int64_t k,
                                                              int64_t id_offset, const Tensor& stats,
                                                              const Tensor& tau) {
  return ip_topk_large_impl(q, p, k, id_offset, stats, tau, true);
}

// global top-k of per-shard canonical lists by exact order key (drt_merge_exact): keys / ids [nparts, nq, k]
std::tuple<Tensor, Tensor> merge_exact(const Tensor& keys_, const Tensor& ids_, int64_t k) {
  need(keys_, "keys", at::kLong, 3);
  need(ids_, "ids", at::kLong, 3);
  TORCH_CHECK_VALUE(keys_.sizes() == ids_.sizes() && keys_.device() == ids_.device(),
                    "merge_exact: keys and ids differ in shape or device");
  TORCH_CHECK_VALUE(keys_.size(2) == k, "merge_exact: lists of ", keys_.size(2), " entries, k = ", k);
  const c10::DeviceGuard g(keys_.device());
  const Tensor keys = keys_.contiguous(), ids = ids_.contiguous();
  const int64_t nq = keys.size(1);
  Tensor s = at::empty({nq, k}, keys.options().dtype(at::kFloat));
  Tensor i = at::empty({nq, k}, keys.options().dtype(at::kLong));
  check_rc(drt_merge_exact((const uint64_t*)keys.data_ptr<int64_t>(), ids.data_ptr<int64_t>(), nq,
                           (int32_t)keys.size(0), (int32_t)k, s.data_ptr<float>(), i.data_ptr<int64_t>(),
                           stream_of(keys)),
           "drt_merge_exact");
  return {s, i};
}

// row statistics of p (+ those of earlier rows in `prev`, appended rows)
Tensor row_stats(const Tensor& p_, const c10::optional<Tensor>& prev) {
  need(p_, "p", at::kBFloat16, 2);
  const c10::DeviceGuard g(p_.device());
  const Tensor p = p_.contiguous();
  Tensor st;
  if (prev.has_value()) {
    stats_ptr(prev, p);
    st = prev->clone();
  } else {
    st = at::empty({DRT_ROW_STATS_LEN}, p.options().dtype(at::kFloat));
  }
  check_rc(drt_row_stats_bf16(p.size(0) ? p.data_ptr() : nullptr, p.size(0), (int32_t)p.size(1),
                              st.data_ptr<float>(), prev.has_value() ? 1 : 0, stream_of(p)),
           "drt_row_stats_bf16");
  return st;
}

// canonical-order stage on a candidate list [nq, kc] (drt_refine_delta_bf16); status updated in place
std::tuple<Tensor, Tensor> refine_delta(const Tensor& q_, const Tensor& p_, int64_t row_offset, const Tensor& cs_,
                                        const Tensor& ci_, int64_t k, const Tensor& stats,
                                        const c10::optional<Tensor>& tau_, Tensor& status, bool local) {
  need(q_, "q", at::kBFloat16, 2);
  need(p_, "p", at::kBFloat16, 2);
  need(cs_, "cand_scores", at::kFloat, 2);
  need(ci_, "cand_ids", at::kLong, 2);
  need(status, "status", at::kInt, 1);
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous(), cs = cs_.contiguous(), ci = ci_.contiguous();
  const int64_t nq = q.size(0), kc = cs.size(1);
  TORCH_CHECK_VALUE(ci.sizes() == cs.sizes() && cs.size(0) == nq, "candidates must be [nq, kc] like q");
  TORCH_CHECK_VALUE(status.is_contiguous() && status.size(0) == nq, "status must be a contiguous [nq] tensor");
  Tensor tau;
  if (tau_.has_value()) {
    need(*tau_, "tau", at::kFloat, 1);
    tau = tau_->contiguous();
    TORCH_CHECK_VALUE(tau.size(0) == nq, "tau must hold one threshold per query");
  }
  Tensor delta = at::empty({nq, kc}, cs.options());
  Tensor cnt = at::empty({nq, 2}, cs.options().dtype(at::kInt));
  // local: every candidate is a row of p (one GPU) -- drt_refine_delta_local_bf16, identical deltas
  check_rc((local ? drt_refine_delta_local_bf16 : drt_refine_delta_bf16)(
               q.data_ptr(), nq, (int32_t)q.size(1), p.size(0) ? p.data_ptr() : nullptr, p.size(0), row_offset,
               cs.data_ptr<float>(), ci.data_ptr<int64_t>(), (int32_t)kc, (int32_t)k, stats_ptr(stats, q),
               tau.defined() ? tau.data_ptr<float>() : nullptr, delta.data_ptr<float>(), cnt.data_ptr<int32_t>(),
               status.data_ptr<int32_t>(), stream_of(q)),
           "drt_refine_delta_bf16");
  return {delta, cnt};
}

std::tuple<Tensor, Tensor> refine_sort(const Tensor& cs_, const Tensor& ci_, const Tensor& delta_, const Tensor& cnt_,
                                       int64_t k) {
  need(cs_, "cand_scores", at::kFloat, 2);
  need(ci_, "cand_ids", at::kLong, 2);
  need(delta_, "delta", at::kFloat, 2);
  need(cnt_, "cnt", at::kInt, 2);
  const c10::DeviceGuard g(cs_.device());
  const Tensor cs = cs_.contiguous(), ci = ci_.contiguous(), delta = delta_.contiguous(), cnt = cnt_.contiguous();
  const int64_t nq = cs.size(0), kc = cs.size(1);
  TORCH_CHECK_VALUE(ci.sizes() == cs.sizes() && delta.sizes() == cs.sizes() && cnt.size(0) == nq,
                    "refine_sort: candidate, delta and cnt shapes disagree");
  Tensor os = at::empty({nq, k}, cs.options());
  Tensor oi = at::empty({nq, k}, ci.options());
  check_rc(drt_refine_sort(cs.data_ptr<float>(), ci.data_ptr<int64_t>(), delta.data_ptr<float>(),
                           cnt.data_ptr<int32_t>(), nq, (int32_t)kc, (int32_t)k, os.data_ptr<float>(),
                           oi.data_ptr<int64_t>(), stream_of(cs)),
           "drt_refine_sort");
  return {os, oi};
}

std::tuple<Tensor, Tensor> topk_merge(const Tensor& scores_, const Tensor& ids_, int64_t k_out) {
  need(scores_, "scores", at::kFloat, 3);
  need(ids_, "ids", at::kLong, 3);
  TORCH_CHECK_VALUE(scores_.sizes() == ids_.sizes(), "topk_merge: scores and ids differ in shape");
  const c10::DeviceGuard g(scores_.device());
  const Tensor s = scores_.contiguous(), i = ids_.contiguous();
  const int64_t nparts = s.size(0), nq = s.size(1), k_in = s.size(2);
  Tensor os = at::empty({nq, k_out}, s.options());
  Tensor oi = at::empty({nq, k_out}, i.options());
  check_rc(drt_topk_merge(s.data_ptr<float>(), i.data_ptr<int64_t>(), nq, (int32_t)nparts, (int32_t)k_in,
                          (int32_t)k_out, os.data_ptr<float>(), oi.data_ptr<int64_t>(), stream_of(s)),
           "drt_topk_merge");
  return {os, oi};
}

Tensor dist_ws(const Tensor& q, int64_t n_local, int64_t n_global, int64_t k, size_t* wsb) {
  *wsb = drt_ip_topk_dist_workspace(q.size(0), n_local, n_global, (int32_t)q.size(1), (int32_t)k);
  TORCH_CHECK_VALUE(*wsb > 0 || q.size(0) == 0, "unsupported dist shape nq=", q.size(0), " n_local=", n_local,
              " n_global=", n_global, " d=", q.size(1), " k=", k);
  return workspace(q, *wsb);
}

Tensor dist_sample(const Tensor& q_, const Tensor& p_, int64_t n_global, int64_t k) {
  need(q_, "q", at::kBFloat16, 2);
  need(p_, "p", at::kBFloat16, 2);
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous();
  const int32_t r = drt_ip_topk_sample_rank((int32_t)k);
  TORCH_CHECK_VALUE(r > 0, "unsupported k=", k);
  Tensor best = at::empty({q.size(0), r}, q.options().dtype(at::kInt));
  size_t wsb = 0;
  Tensor ws = dist_ws(q, p.size(0), n_global, k, &wsb);
  check_rc(drt_ip_topk_dist_sample(q.data_ptr(), q.size(0), p.size(0) ? p.data_ptr() : nullptr, p.size(0), n_global,
                                   (int32_t)q.size(1), (int32_t)k, (uint32_t*)best.data_ptr<int32_t>(), ws.data_ptr(),
                                   wsb, stream_of(q)),
           "drt_ip_topk_dist_sample");
  return best;
}

Tensor dist_tau(const Tensor& lists_, int64_t k) {
  need(lists_, "lists", at::kInt, 3);
  const c10::DeviceGuard g(lists_.device());
  const Tensor lists = lists_.contiguous();
  Tensor tau = at::empty({lists.size(1)}, lists.options().dtype(at::kFloat));
  check_rc(drt_ip_topk_dist_tau((const uint32_t*)lists.data_ptr<int32_t>(), lists.size(1), (int32_t)lists.size(0),
                                (int32_t)k, tau.data_ptr<float>(), stream_of(lists)),
           "drt_ip_topk_dist_tau");
  return tau;
}

Tensor dist_filter(const Tensor& q_, const Tensor& p_, int64_t n_global, int64_t k, int64_t id_offset,
                   const Tensor& tau_) {
  need(q_, "q", at::kBFloat16, 2);
  need(p_, "p", at::kBFloat16, 2);
  need(tau_, "tau", at::kFloat, 1);
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous(), tau = tau_.contiguous();
  Tensor packed = at::empty({q.size(0), k + 1}, q.options().dtype(at::kLong));
  size_t wsb = 0;
  Tensor ws = dist_ws(q, p.size(0), n_global, k, &wsb);
  check_rc(drt_ip_topk_dist_filter(q.data_ptr(), q.size(0), p.size(0) ? p.data_ptr() : nullptr, p.size(0), n_global,
                                   (int32_t)q.size(1), (int32_t)k, id_offset, tau.data_ptr<float>(),
                                   (uint64_t*)packed.data_ptr<int64_t>(), ws.data_ptr(), wsb, stream_of(q)),
           "drt_ip_topk_dist_filter");
  return packed;
}

Tensor dist_filter_lists(const Tensor& q_, const Tensor& p_, int64_t n_global, int64_t k, int64_t id_offset,
                         const Tensor& lists_) {
  need(q_, "q", at::kBFloat16, 2);
  need(p_, "p", at::kBFloat16, 2);
  need(lists_, "lists", at::kInt, 3);
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous(), lists = lists_.contiguous();
  TORCH_CHECK_VALUE(lists.size(1) == q.size(0), "lists must be [nlists, nq, r]");
  Tensor packed = at::empty({q.size(0), k + 1}, q.options().dtype(at::kLong));
  size_t wsb = 0;
  Tensor ws = dist_ws(q, p.size(0), n_global, k, &wsb);
  check_rc(drt_ip_topk_dist_filter_lists(q.data_ptr(), q.size(0), p.size(0) ? p.data_ptr() : nullptr, p.size(0),
                                         n_global, (int32_t)q.size(1), (int32_t)k, id_offset,
                                         (const uint32_t*)lists.data_ptr<int32_t>(), (int32_t)lists.size(0), nullptr,
                                         (uint64_t*)packed.data_ptr<int64_t>(), ws.data_ptr(), wsb, stream_of(q)),
           "drt_ip_topk_dist_filter_lists");
  return packed;
}

// dist_filter writing into `packed` ([nq, k + 1] contiguous, e.g. a row slice of a group buffer); tau is
// this batch's [nq] slice of a group's thresholds.
void dist_filter_into(const Tensor& q_, const Tensor& p_, int64_t n_global, int64_t k, int64_t id_offset,
                      const Tensor& tau_, Tensor& packed) {
  need(q_, "q", at::kBFloat16, 2);
  need(p_, "p", at::kBFloat16, 2);
  need(tau_, "tau", at::kFloat, 1);
  need(packed, "packed", at::kLong, 2);
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous(), tau = tau_.contiguous();
  TORCH_CHECK_VALUE(tau.size(0) == q.size(0), "tau must hold one threshold per query");
  TORCH_CHECK_VALUE(packed.is_contiguous() && packed.size(0) == q.size(0) && packed.size(1) == k + 1,
                    "packed must be a contiguous [nq, k + 1] tensor");
  size_t wsb = 0;
  Tensor ws = dist_ws(q, p.size(0), n_global, k, &wsb);
  check_rc(drt_ip_topk_dist_filter(q.data_ptr(), q.size(0), p.size(0) ? p.data_ptr() : nullptr, p.size(0), n_global,
                                   (int32_t)q.size(1), (int32_t)k, id_offset, tau.data_ptr<float>(),
                                   (uint64_t*)packed.data_ptr<int64_t>(), ws.data_ptr(), wsb, stream_of(q)),
           "drt_ip_topk_dist_filter");
}

// dist_filter over the shard in row chunks (chunk c = rows [starts[c], starts[c + 1])): one scan launch per
// chunk, one hit list and one select -- the same packed lists as dist_filter_into over the whole shard.
void dist_filter_chunks_into(const Tensor& q_, const Tensor& p_, int64_t n_global, int64_t k, int64_t id_offset,
                             const Tensor& tau_, at::IntArrayRef starts, Tensor& packed) {
  need(q_, "q", at::kBFloat16, 2);
  need(p_, "p", at::kBFloat16, 2);
  need(tau_, "tau", at::kFloat, 1);
  need(packed, "packed", at::kLong, 2);
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous(), tau = tau_.contiguous();
  TORCH_CHECK_VALUE(tau.size(0) == q.size(0), "tau must hold one threshold per query");
  TORCH_CHECK_VALUE(packed.is_contiguous() && packed.size(0) == q.size(0) && packed.size(1) == k + 1,
                    "packed must be a contiguous [nq, k + 1] tensor");
  TORCH_CHECK_VALUE(starts.size() >= 2 && starts.front() == 0 && starts.back() == p.size(0),
                    "starts must run from 0 to the shard's row count");
  for (size_t c = 1; c < starts.size(); ++c) TORCH_CHECK_VALUE(starts[c - 1] <= starts[c], "starts must not decrease");
  TORCH_CHECK_VALUE(q.size(1) <= 768, "chunked filtering takes d <= 768");
  size_t wsb = 0;
  Tensor ws = dist_ws(q, p.size(0), n_global, k, &wsb);
  const std::vector<int64_t> st(starts.begin(), starts.end());
  check_rc(drt_ip_topk_dist_filter_chunks(q.data_ptr(), q.size(0), p.size(0) ? p.data_ptr() : nullptr, p.size(0),
                                          n_global, (int32_t)q.size(1), (int32_t)k, id_offset,
                                          tau.data_ptr<float>(), (uint64_t*)packed.data_ptr<int64_t>(), st.data(),
                                          (int32_t)st.size() - 1, ws.data_ptr(), wsb, stream_of(q)),
           "drt_ip_topk_dist_filter_chunks");
}

// dist_filter_lists for query rows [q0, q0 + nq) of lists [nlists, NQ, r] gathered for a group of
// batches, writing the packed lists into `packed` ([nq, k + 1], e.g. a row slice of a group buffer).
void dist_filter_lists_into(const Tensor& q_, const Tensor& p_, int64_t n_global, int64_t k, int64_t id_offset,
                            const Tensor& lists, int64_t q0, Tensor& packed) {
  need(q_, "q", at::kBFloat16, 2);
  need(p_, "p", at::kBFloat16, 2);
  need(lists, "lists", at::kInt, 3);
  need(packed, "packed", at::kLong, 2);
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous();
  TORCH_CHECK_VALUE(lists.is_contiguous(), "lists must be a contiguous [nlists, NQ, r] tensor");
  TORCH_CHECK_VALUE(q0 >= 0 && q0 + q.size(0) <= lists.size(1), "query rows [", q0, ", ", q0 + q.size(0),
                    ") outside the lists' ", lists.size(1), " rows");
  TORCH_CHECK_VALUE(packed.is_contiguous() && packed.size(0) == q.size(0) && packed.size(1) == k + 1,
                    "packed must be a contiguous [nq, k + 1] tensor");
  const int64_t r = lists.size(2);
  TORCH_CHECK_VALUE(r == drt_ip_topk_sample_rank((int32_t)k), "lists hold ", r, " keys per query, k=", k, " needs ",
                    drt_ip_topk_sample_rank((int32_t)k));
  size_t wsb = 0;
  Tensor ws = dist_ws(q, p.size(0), n_global, k, &wsb);
  check_rc(drt_ip_topk_dist_filter_lists_at(q.data_ptr(), q.size(0), p.size(0) ? p.data_ptr() : nullptr, p.size(0),
                                            n_global, (int32_t)q.size(1), (int32_t)k, id_offset,
                                            (const uint32_t*)lists.data_ptr<int32_t>() + q0 * r,
                                            (int32_t)lists.size(0), lists.size(1) * r, nullptr,
                                            (uint64_t*)packed.data_ptr<int64_t>(), ws.data_ptr(), wsb, stream_of(q)),
           "drt_ip_topk_dist_filter_lists_at");
}

std::tuple<Tensor, Tensor, Tensor> merge_packed(const Tensor& parts_, int64_t k, int64_t n_global, int64_t k_cert) {
  need(parts_, "parts", at::kLong, 3);
  TORCH_CHECK_VALUE(parts_.size(2) >= 2 && parts_.size(2) <= k + 1,
                    "merge_packed expects [nparts, nq, lcap + 1] lists with lcap <= k");
  const c10::DeviceGuard g(parts_.device());
  const Tensor parts = parts_.contiguous();
  const int64_t nq = parts.size(1), lcap = parts.size(2) - 1;
  Tensor s = at::empty({nq, k}, parts.options().dtype(at::kFloat));
  Tensor i = at::empty({nq, k}, parts.options().dtype(at::kLong));
  Tensor st = at::empty({nq}, parts.options().dtype(at::kInt));
  if (lcap < k) {   // capped exchange lists (drt_topk_merge_packed_capped)
    check_rc(drt_topk_merge_packed_capped((const uint64_t*)parts.data_ptr<int64_t>(), nq, (int32_t)parts.size(0),
                                          (int32_t)lcap, (int32_t)k, (int32_t)(k_cert > 0 ? k_cert : k), n_global,
                                          s.data_ptr<float>(), i.data_ptr<int64_t>(), st.data_ptr<int32_t>(),
                                          stream_of(parts)),
             "drt_topk_merge_packed_capped");
    return {s, i, st};
  }
  check_rc(drt_topk_merge_packed_cert((const uint64_t*)parts.data_ptr<int64_t>(), nq, (int32_t)parts.size(0),
                                      (int32_t)k, (int32_t)(k_cert > 0 ? k_cert : k), n_global, s.data_ptr<float>(),
                                      i.data_ptr<int64_t>(), st.data_ptr<int32_t>(), stream_of(parts)),
           "drt_topk_merge_packed_cert");
  return {s, i, st};
}

// ---------------------------------------------------------------------------- training loss
std::tuple<Tensor, Tensor, Tensor> score_ce_fwd(const Tensor& q_, const Tensor& p_, int64_t target_stride,
                                                double scale) {
  need(q_, "q", at::kFloat, 2);
  need(p_, "p", at::kFloat, 2);
  TORCH_CHECK_VALUE(q_.size(1) == p_.size(1), "q ", q_.sizes(), " and p ", p_.sizes(), " differ in dimension");
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous();
  const int64_t m = q.size(0), n = p.size(0), d = q.size(1);
  Tensor S = at::empty({m, n}, q.options());
  Tensor lse = at::empty({m}, q.options());
  Tensor loss = at::empty({}, q.options());
  const size_t wsb = drt_score_ce_workspace(m, n, (int32_t)d);
  Tensor ws = workspace(q, wsb);
  check_rc(drt_score_ce_fwd(q.data_ptr<float>(), p.data_ptr<float>(), m, n, (int32_t)d, target_stride, (float)scale,
                            S.data_ptr<float>(), lse.data_ptr<float>(), loss.data_ptr<float>(), ws.data_ptr(), wsb,
                            stream_of(q)),
           "drt_score_ce_fwd");
  return {loss, S, lse};
}

std::tuple<Tensor, Tensor> score_ce_bwd(const Tensor& grad_, const Tensor& q_, const Tensor& p_, const Tensor& S_,
                                        const Tensor& lse_, int64_t target_stride, double scale) {
  need(q_, "q", at::kFloat, 2);
  need(p_, "p", at::kFloat, 2);
  need(S_, "scores", at::kFloat, 2);
  need(lse_, "lse", at::kFloat, 1);
  const c10::DeviceGuard g(q_.device());
  const Tensor q = q_.contiguous(), p = p_.contiguous(), S = S_.contiguous(), lse = lse_.contiguous();
  const Tensor grad = grad_.to(at::kFloat).contiguous().reshape({1});
  const int64_t m = q.size(0), n = p.size(0), d = q.size(1);
  Tensor dq = at::empty({m, d}, q.options());
  Tensor dp = at::empty({n, d}, q.options());
  const size_t wsb = drt_score_ce_workspace(m, n, (int32_t)d);
  Tensor ws = workspace(q, wsb);
  check_rc(drt_score_ce_bwd(q.data_ptr<float>(), p.data_ptr<float>(), S.data_ptr<float>(), lse.data_ptr<float>(), m,
                            n, (int32_t)d, target_stride, grad.data_ptr<float>(), (float)scale, dq.data_ptr<float>(),
                            dp.data_ptr<float>(), ws.data_ptr(), wsb, stream_of(q)),
           "drt_score_ce_bwd");
  return {dq, dp};
}

// ---------------------------------------------------------------------------- encoder pieces
Tensor embed_ln(const Tensor& ids_, const c10::optional<Tensor>& type_ids, const Tensor& word, const Tensor& pos,
                const Tensor& type, const Tensor& gamma, const Tensor& beta, double eps) {
  need(ids_, "input_ids", at::kLong, 2);
  const c10::DeviceGuard g(ids_.device());
  const Tensor ids = ids_.contiguous();
  const int64_t B = ids.size(0), L = ids.size(1), H = word.size(1);
  TORCH_CHECK(L <= pos.size(0), "sequence length ", L, " exceeds max_position_embeddings ", pos.size(0));
  c10::optional<Tensor> tt;
  if (type_ids.has_value()) tt = type_ids->contiguous();
  Tensor out = at::empty({B, L, H}, ids.options().dtype(at::kBFloat16));
  check_rc(drt_embed_ln(ids.data_ptr<int64_t>(), tt.has_value() ? tt->data_ptr<int64_t>() : nullptr, B, L,
                        word.data_ptr<float>(), pos.data_ptr<float>(), type.data_ptr<float>(), gamma.data_ptr<float>(),
                        beta.data_ptr<float>(), (float)eps, (int32_t)H, out.data_ptr(), stream_of(ids)),
           "drt_embed_ln");
  return out;
}

Tensor linear(const Tensor& x_, const Tensor& w_, const c10::optional<Tensor>& bias,
              const c10::optional<Tensor>& residual, bool gelu, bool fp32_out) {
  need(x_, "x", at::kBFloat16, 2);
  need(w_, "w", at::kBFloat16, 2);
  TORCH_CHECK(x_.size(1) == w_.size(1), "linear: x ", x_.sizes(), " and w ", w_.sizes(), " differ in K");
  const c10::DeviceGuard g(x_.device());
  const Tensor x = x_.contiguous(), w = w_.contiguous();
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  if (bias.has_value()) TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == N, "bias: float [N]");
  c10::optional<Tensor> res;
  if (residual.has_value()) {
    TORCH_CHECK(residual->scalar_type() == at::kBFloat16 && residual->numel() == M * N, "residual: bf16 [M, N]");
    res = residual->contiguous();
  }
  Tensor y = at::empty({M, N}, x.options().dtype(fp32_out ? at::kFloat : at::kBFloat16));
  const int32_t flags = (gelu ? 1 : 0) | (fp32_out ? 2 : 0);
  const size_t wsb = drt_linear_workspace(M, N, K);
  Tensor ws = workspace(x, wsb);
  check_rc(drt_linear_bf16_ws(x.data_ptr(), w.data_ptr(), bias.has_value() ? bias->data_ptr<float>() : nullptr,
                              res.has_value() ? res->data_ptr() : nullptr, y.data_ptr(), M, N, K, flags,
                              wsb ? ws.data_ptr() : nullptr, wsb, stream_of(x)),
           "drt_linear_bf16_ws");
  return y;
}

Tensor attention(const Tensor& qkv_, const c10::optional<Tensor>& mask, int64_t B, int64_t heads, double scale) {
  need(qkv_, "qkv", at::kBFloat16, 2);
  const c10::DeviceGuard g(qkv_.device());
  const Tensor qkv = qkv_.contiguous();
  const int64_t T = qkv.size(0), H3 = qkv.size(1);
  TORCH_CHECK(B > 0 && T % B == 0 && H3 % (3 * heads) == 0, "attention: qkv must be [B*L, 3*heads*64]");
  const int64_t L = T / B, hd = H3 / (3 * heads);
  c10::optional<Tensor> m;
  if (mask.has_value()) {
    TORCH_CHECK(mask->numel() == B * L, "attention: mask must be [B, L]");
    m = mask->to(at::kLong).contiguous();
  }
  Tensor ctx = at::empty({T, heads * hd}, qkv.options());
  check_rc(drt_attention_bf16(qkv.data_ptr(), m.has_value() ? m->data_ptr<int64_t>() : nullptr, ctx.data_ptr(), B, L,
                              (int32_t)heads, (int32_t)hd, (float)scale, stream_of(qkv)),
           "drt_attention_bf16");
  return ctx;
}

Tensor layernorm(const Tensor& x_, const Tensor& gamma, const Tensor& beta, double eps) {
  need_gpu(x_, "x");
  const c10::DeviceGuard g(x_.device());
  const Tensor x = x_.contiguous();
  const int64_t H = x.size(-1), M = x.numel() / H;
  Tensor out = at::empty(x.sizes(), x.options().dtype(at::kBFloat16));
  int rc;
  if (x.scalar_type() == at::kFloat)
    rc = drt_layernorm_f32_bf16(x.data_ptr<float>(), M, (int32_t)H, gamma.data_ptr<float>(), beta.data_ptr<float>(),
                                (float)eps, out.data_ptr(), stream_of(x));
  else {
    TORCH_CHECK(x.scalar_type() == at::kBFloat16, "layernorm: x must be float or bfloat16");
    rc = drt_layernorm_bf16(x.data_ptr(), M, (int32_t)H, gamma.data_ptr<float>(), beta.data_ptr<float>(), (float)eps,
                            out.data_ptr(), stream_of(x));
  }
  check_rc(rc, "drt_layernorm");
  return out;
}

Tensor pool(const Tensor& hidden_, const c10::optional<Tensor>& mask, int64_t mode) {
  need(hidden_, "hidden", at::kBFloat16, 3);
  const c10::DeviceGuard g(hidden_.device());
  const Tensor hidden = hidden_.contiguous();
  const int64_t B = hidden.size(0), L = hidden.size(1), H = hidden.size(2);
  c10::optional<Tensor> m;
  if (mask.has_value()) m = mask->to(at::kLong).contiguous();
  Tensor reps = at::empty({B, H}, hidden.options().dtype(at::kFloat));
  check_rc(drt_pool_bf16(hidden.data_ptr(), m.has_value() ? m->data_ptr<int64_t>() : nullptr, B, L, (int32_t)H,
                         (int32_t)mode, reps.data_ptr<float>(), nullptr, stream_of(hidden)),
           "drt_pool_bf16");
  return reps;
}

Tensor l2_normalize(const Tensor& x_) {
  need(x_, "x", at::kFloat, 2);
  const c10::DeviceGuard g(x_.device());
  Tensor x = x_.clone(at::MemoryFormat::Contiguous);
  check_rc(drt_l2_normalize_f32(x.data_ptr<float>(), x.size(0), (int32_t)x.size(1), nullptr, stream_of(x)),
           "drt_l2_normalize_f32");
  return x;
}

}  // namespace

TORCH_LIBRARY(drt, m) {
  m.def("ip_topk(Tensor q, Tensor p, int k, int id_offset=0, Tensor? stats=None) -> (Tensor, Tensor, Tensor)");
  m.def("ip_topk.out(Tensor q, Tensor p, int k, int id_offset, Tensor? stats=None, *, Tensor(a!) scores, "
        "Tensor(b!) ids, Tensor(c!) status) -> ()");
  m.def("ip_topk_resolve(Tensor q, Tensor p, int k, int id_offset, Tensor(a!) scores, Tensor(b!) ids, "
        "Tensor(c!) status, Tensor? stats=None) -> int");
  m.def("ip_topk_resolve_wide(Tensor q, Tensor p, int k, int id_offset, Tensor(a!) scores, Tensor(b!) ids, "
        "Tensor(c!) status, Tensor stats) -> int");
  m.def("ip_topk_large(Tensor q, Tensor p, int k, int id_offset, Tensor stats, Tensor tau) -> (Tensor, Tensor, Tensor)");
  m.def("ip_topk_large_keys(Tensor q, Tensor p, int k, int id_offset, Tensor stats, Tensor tau) -> "
        "(Tensor, Tensor, Tensor, Tensor)");
  m.def("merge_exact(Tensor keys, Tensor ids, int k) -> (Tensor, Tensor)");
  m.def("row_stats(Tensor p, Tensor? prev=None) -> Tensor");
  m.def("refine_delta(Tensor q, Tensor p, int row_offset, Tensor cand_scores, Tensor cand_ids, int k, Tensor stats, "
        "Tensor? tau, Tensor(a!) status, bool local=False) -> (Tensor, Tensor)");
  m.def("refine_sort(Tensor cand_scores, Tensor cand_ids, Tensor delta, Tensor cnt, int k) -> (Tensor, Tensor)");
  m.def("topk_merge(Tensor scores, Tensor ids, int k_out) -> (Tensor, Tensor)");
  m.def("dist_sample(Tensor q, Tensor p, int n_global, int k) -> Tensor");
  m.def("dist_tau(Tensor lists, int k) -> Tensor");
  m.def("dist_filter(Tensor q, Tensor p, int n_global, int k, int id_offset, Tensor tau) -> Tensor");
  m.def("dist_filter_lists(Tensor q, Tensor p, int n_global, int k, int id_offset, Tensor lists) -> Tensor");
  m.def("dist_filter_lists_into(Tensor q, Tensor p, int n_global, int k, int id_offset, Tensor lists, int q0, "
        "Tensor(a!) packed) -> ()");
  m.def("dist_filter_into(Tensor q, Tensor p, int n_global, int k, int id_offset, Tensor tau, Tensor(a!) packed) -> ()");
  m.def("dist_filter_chunks_into(Tensor q, Tensor p, int n_global, int k, int id_offset, Tensor tau, int[] starts, "
        "Tensor(a!) packed) -> ()");
  m.def("merge_packed(Tensor parts, int k, int n_global, int k_cert=-1) -> (Tensor, Tensor, Tensor)");
  m.def("score_ce_fwd(Tensor q, Tensor p, int target_stride, float scale) -> (Tensor, Tensor, Tensor)");
  m.def("score_ce_bwd(Tensor grad, Tensor q, Tensor p, Tensor scores, Tensor lse, int target_stride, "
        "float scale) -> (Tensor, Tensor)");
  m.def("embed_ln(Tensor input_ids, Tensor? token_type_ids, Tensor word, Tensor pos, Tensor type, Tensor gamma, "
        "Tensor beta, float eps) -> Tensor");
  m.def("linear(Tensor x, Tensor w, Tensor? bias, Tensor? residual, bool gelu=False, bool fp32_out=False) -> Tensor");
  m.def("attention(Tensor qkv, Tensor? mask, int batch, int heads, float scale) -> Tensor");
  m.def("layernorm(Tensor x, Tensor gamma, Tensor beta, float eps) -> Tensor");
  m.def("pool(Tensor hidden, Tensor? mask, int mode) -> Tensor");
  m.def("l2_normalize(Tensor x) -> Tensor");
}

TORCH_LIBRARY_IMPL(drt, CUDA, m) {   // the GPU dispatch key of torch-ROCm
  m.impl("ip_topk", &ip_topk);
  m.impl("ip_topk.out", &ip_topk_out);
  m.impl("dist_filter_chunks_into", &dist_filter_chunks_into);
  m.impl("ip_topk_resolve", &ip_topk_resolve);
  m.impl("ip_topk_resolve_wide", &ip_topk_resolve_wide);
  m.impl("ip_topk_large", &ip_topk_large);
  m.impl("ip_topk_large_keys", &ip_topk_large_keys);
  m.impl("merge_exact", &merge_exact);
  m.impl("row_stats", &row_stats);
  m.impl("refine_delta", &refine_delta);
  m.impl("refine_sort", &refine_sort);
  m.impl("topk_merge", &topk_merge);
  m.impl("dist_sample", &dist_sample);
  m.impl("dist_tau", &dist_tau);
  m.impl("dist_filter", &dist_filter);
  m.impl("dist_filter_lists", &dist_filter_lists);
  m.impl("dist_filter_lists_into", &dist_filter_lists_into);
  m.impl("dist_filter_into", &dist_filter_into);
  m.impl("merge_packed", &merge_packed);
  m.impl("score_ce_fwd", &score_ce_fwd);
  m.impl("score_ce_bwd", &score_ce_bwd);
  m.impl("embed_ln", &embed_ln);
  m.impl("linear", &linear);
  m.impl("attention", &attention);
  m.impl("layernorm", &layernorm);
  m.impl("pool", &pool);
  m.impl("l2_normalize", &l2_normalize);
}
