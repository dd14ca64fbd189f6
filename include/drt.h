/*
 * drt.h — C ABI of the MI355X-native dense-retrieval hot path.
 *
 * This is the drop-in boundary BELOW the reference's Python classes.  The
 * reference (yhao-wang/DenseRetrievalToolkits) has no native layer of its own:
 * its arithmetic sits in third-party code reached from these Python sites,
 * which the entry points below replace one for one:
 *
 *   faiss.IndexFlatIP.add/search        DRT/evaluator/index.py:16-33
 *       -> drt_ip_topk_bf16 / drt_ip_topk_resolve (per row shard)
 *   partition merge (utils.py:215-229, trainer.py:220-262 file exchange)
 *       -> drt_topk_merge
 *   torch.matmul(q, p.T) score matrix    DRT/model/biencoder.py:107,
 *                                        DRT/trainer/losses.py:16
 *       -> drt_gemm_nt_bf16 (fp32 scores)
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer owned by the caller; nothing is
 *     allocated inside the asynchronous entry points (workspace is sized by the
 *     *_workspace query and passed in);
 *   - work is enqueued on `stream` (a hipStream_t passed as void*); the call
 *     returns after enqueueing;
 *   - return value: 0 = DRT_OK, DRT_EINVAL (-1) for a bad argument, otherwise
 *     the hipError_t of the failing HIP call;
 *   - bf16 tensors are row-major with unit stride in the last dimension and
 *     16-byte aligned rows.
 *   - result order is (score descending, id ascending): the reference sorts
 *     by -score with an unspecified tie order (index.py:33); the build pins
 *     ties to ascending id.  Rows past the available hits are padded with
 *     id -1 and score -FLT_MAX (faiss IndexFlatIP convention).
 */
#ifndef DRT_H_
#define DRT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DRT_OK 0
#define DRT_EINVAL (-1)
#define DRT_ROW_STATS_LEN 34   /* floats of drt_row_stats_bf16's statistics (2 + 32 k-steps) */

/* Library version / self-description (host only, no GPU needed). */
const char* drt_version(void);

/* ------------------------------------------------------------------------
 * Brute-force inner-product top-k over one row shard  (index.py:16-33)
 * ------------------------------------------------------------------------
 * Q: [nq, d] bf16 queries.  P: [n, d] bf16 corpus shard (row i has global id
 * id_offset + i).  d must be a multiple of 64 and <= 1024 (FlatIPIndex zero-pads any other d <= 1024); 1 <= k <= 2048.
 * Writes out_scores [nq, k] fp32 and out_ids [nq, k] int64, and status [nq]
 * int32: 0 = exact result, 1 = the fast threshold path could not certify the
 * query and drt_ip_topk_resolve must be called for it (probability ~1e-9 per
 * query on non-degenerate data).                             */
size_t drt_ip_topk_workspace(int64_t nq, int64_t n, int32_t d, int32_t k);
int drt_ip_topk_bf16(const void* Q, int64_t nq, const void* P, int64_t n, int32_t d,
                     int32_t k, int64_t id_offset, float* out_scores, int64_t* out_ids,
                     int32_t* status, void* workspace, size_t workspace_bytes,
                     void* stream);

/* Exact slow path for every query whose status (device array from
 * drt_ip_topk_bf16) is non-zero.  SYNCHRONOUS: reads status back, rescans the
 * shard for those queries only (dense scores of up to ~2 GB per chunk in the
 * caller's workspace: drt_ip_topk_resolve_workspace(#failed queries, n, d)
 * bytes; a smaller workspace means smaller chunks, too small = DRT_EINVAL),
 * and clears their status.  Returns the number of resolved queries in
 * *n_resolved (may be NULL).  Nothing is allocated inside.                  */
size_t drt_ip_topk_resolve_workspace(int64_t n_failed, int64_t n, int32_t d);
int drt_ip_topk_resolve(const void* Q, int64_t nq, const void* P, int64_t n, int32_t d,
                        int32_t k, int64_t id_offset, float* out_scores, int64_t* out_ids,
                        int32_t* status, void* workspace, size_t workspace_bytes,
                        int64_t* n_resolved, void* stream);

/* ------------------------------------------------------------------------
 * Canonical (exact-score) order  (the fp64 evaluator's answer)
 * ------------------------------------------------------------------------
 * The scan ranks rows by fp32 sums of the bf16 products; rows whose exact inner products lie
 * within the fp32 summation error of each other (or of the k-th score) may come out in either
 * order.  These entry points put a result in the order of the EXACT products (fp64 sums of the
 * bf16 products, ties by ascending id), as an fp64 CPU evaluator (faiss's semantics without its
 * rounding) ranks them, with scores = the exact sums rounded to fp32.
 * drt_row_stats_bf16: stats[DRT_ROW_STATS_LEN] (device floats) = (max squared L2 norm over the rows,
 *   1.0f while every element is an integer, then for each 32-element k-step t < ceil(d / 32) the max
 *   over the rows of the squared norm of the prefix [0, 32 (t + 1))) -- the error bound of the scan's
 *   MFMA chain (csrc/search.hip, "Error bound"); accumulate = 0 (re)initialises, 1 combines with the
 *   stats already there (appended rows).  Across shards combine by max (the flag by min).  Reads
 *   every row once.  d <= 1024.
 * drt_ip_topk_exact_bf16: drt_ip_topk_bf16 in the canonical order (same workspace).  status bit 0
 *   as drt_ip_topk_bf16 (call drt_ip_topk_resolve_exact); bit 1 = the exact order could not be
 *   certified from the candidate list and the query holds the (exact) fp32 top-k in the fp32 order:
 *   more than drt_refine_width(k) - k rows within the fp32 error of the k-th score, or that window
 *   reaching below the filter threshold (massive near-ties) -- call drt_ip_topk_resolve_wide.
 * drt_ip_topk_resolve_exact: drt_ip_topk_resolve in the canonical order (status bit 0 only).
 * drt_ip_topk_resolve_wide: SYNCHRONOUS, for the queries whose status is exactly 2: a filter pass at
 *   the lowered threshold s_k - 2 eps collects every row that may belong to the exact top-k (up to
 *   65536 per query), their exact sums are computed and the top-k by (exact score desc, id asc) is
 *   written in place; bit 1 is cleared for every such query whose collected set fit.  Workspace:
 *   drt_ip_topk_resolve_wide_workspace(n, d) bytes (~134 MB, chunks of 128 queries).
 * drt_refine_delta_bf16 / drt_refine_sort: the stage alone, on a candidate list cand [nq][kc]
 *   (scores desc, global ids, kc = drt_refine_width(k), e.g. a merged sharded result): delta =
 *   exact - fp32 score for the candidates whose rows this shard holds (row_offset = global id of
 *   its row 0; 0 elsewhere, so shards combine their deltas with one SUM all-reduce), cnt [nq][2]
 *   (window size, eps) per query; then the sort writes the top-k.  tau [nq] = the filter thresholds the
 *   candidate list was collected with (NULL: every row was scored).                           */
int drt_row_stats_bf16(const void* P, int64_t n, int32_t d, float* stats, int32_t accumulate, void* stream);
int32_t drt_refine_width(int32_t k);
int drt_ip_topk_exact_bf16(const void* Q, int64_t nq, const void* P, int64_t n, int32_t d, int32_t k,
                           int64_t id_offset, const float* stats, float* out_scores, int64_t* out_ids,
                           int32_t* status, void* workspace, size_t workspace_bytes, void* stream);
int drt_ip_topk_resolve_exact(const void* Q, int64_t nq, const void* P, int64_t n, int32_t d, int32_t k,
                              int64_t id_offset, const float* stats, float* out_scores, int64_t* out_ids,
                              int32_t* status, void* workspace, size_t workspace_bytes, int64_t* n_resolved,
                              void* stream);
size_t drt_ip_topk_resolve_wide_workspace(int64_t n, int32_t d);
int drt_ip_topk_resolve_wide(const void* Q, int64_t nq, const void* P, int64_t n, int32_t d, int32_t k,
                             int64_t id_offset, const float* stats, float* out_scores, int64_t* out_ids,
                             int32_t* status, void* workspace, size_t workspace_bytes, int64_t* n_resolved,
                             void* stream);
/* drt_ip_topk_large: top-k for 2048 < k <= 32768 (faiss IndexFlatIP answers any k; the reference's
 *   retrieve_num is a free flag, DRT/arguments.py:195 used at DRT/trainer/trainer.py:296-297, searched
 *   through DRT/evaluator/index.py:31-33), always in the canonical order (exact score desc, id asc;
 *   scores = exact sums rounded to fp32; rows past n padded with -1 like drt_ip_topk_bf16).  tau [nq]
 *   = a lower bound of each query's k-th fp32 scan score, e.g. the minimum over C disjoint row ranges
 *   of their m-th score with C * m >= k (-inf: every row).  Every row with fp32 score >= tau - 2 eps
 *   is collected (up to 65536 per query) and ranked by its exact sum.  Asynchronous; status 0, or 2
 *   where the collected set overflowed (that query's output is then undefined).  Workspace:
 *   drt_ip_topk_large_workspace(d, k) bytes (0 = unsupported d / k).                            */
size_t drt_ip_topk_large_workspace(int32_t d, int32_t k);
int drt_ip_topk_large(const void* Q, int64_t nq, const void* P, int64_t n, int32_t d, int32_t k, int64_t id_offset,
                      const float* stats, const float* tau, float* out_scores, int64_t* out_ids, int32_t* status,
                      void* workspace, size_t workspace_bytes, void* stream);
/* The same, also writing each output entry's EXACT order key (u64 [nq, k]: ascending = exact score desc;
 * ~0 for pads) -- the per-shard step of a sharded search at k > 2048 (round 6), merged across shards by
 * drt_merge_exact after an all-gather of (keys, global ids).                                            */
int drt_ip_topk_large_keys(const void* Q, int64_t nq, const void* P, int64_t n, int32_t d, int32_t k,
                           int64_t id_offset, const float* stats, const float* tau, float* out_scores,
                           int64_t* out_ids, uint64_t* out_keys, int32_t* status, void* workspace,
                           size_t workspace_bytes, void* stream);
/* drt_merge_exact: the global top-k of nparts per-shard canonical lists ([nparts][nq][k] exact order keys
 *   + global ids, each sorted by (key, id), pads (~0, -1) last) by (exact key, id) -- the reference's
 *   partition merge (merge_retrieval_results_by_score, DRT/model/utils.py:215-229) on exact scores;
 *   out_scores = the exact sums rounded to fp32, missing entries (-FLT_MAX, -1).  Asynchronous.          */
int drt_merge_exact(const uint64_t* keys, const int64_t* ids, int64_t nq, int32_t nparts, int32_t k,
                    float* out_scores, int64_t* out_ids, void* stream);
int drt_refine_delta_bf16(const void* Q, int64_t nq, int32_t d, const void* P, int64_t n_local,
                          int64_t row_offset, const float* cand_s, const int64_t* cand_i, int32_t kc,
                          int32_t k, const float* stats, const float* tau, float* delta, int32_t* cnt,
                          int32_t* status, void* stream);
/* The same for an index whose single shard holds every candidate (one GPU): identical deltas, the
 * exact sums computed by waves walking the window directly instead of compacting owned rows. */
int drt_refine_delta_local_bf16(const void* Q, int64_t nq, int32_t d, const void* P, int64_t n_local,
                                int64_t row_offset, const float* cand_s, const int64_t* cand_i, int32_t kc,
                                int32_t k, const float* stats, const float* tau, float* delta, int32_t* cnt,
                                int32_t* status, void* stream);
int drt_refine_sort(const float* cand_s, const int64_t* cand_i, const float* delta, const int32_t* cnt,
                    int64_t nq, int32_t kc, int32_t k, float* out_scores, int64_t* out_ids, void* stream);

/* Answer matching of retrieved passages (has_answers, DRT/evaluator/nq_eval.py:187-218) on token ids
 * resident in HBM: tok [slots][W] int32 (-1 pads; evaluator/nq_eval.py RowAnswerMatcher), rows [B][k]
 * int64 = the retrieved index rows (-1: pad -> 0), slot_of [n_rows] int64 = each row's token slot (-1:
 * not tokenised -> 0; slot_of NULL: rows already hold slots), ans [B][A][n_max] int32 + alen [B][A]
 * (the answers' token ids; alen 0 = no answer), every [B] (1: an empty answer, every passage matches).
 * hit [B][k] int8 = 1 iff some answer occurs as a contiguous token window.                      */
int drt_answer_match_i32(const int32_t* tok, int32_t W, const int64_t* rows, const int64_t* slot_of, int64_t n_rows,
                         int64_t B, int64_t k, const int32_t* ans, const int32_t* alen, int32_t A, int32_t n_max,
                         const uint8_t* every, int8_t* hit, void* stream);

/* get_metrics (DRT/evaluator/metrics.py:4-59) of one loader batch's hit matrix hit [B][k] (int8, from
 * drt_answer_match_i32), ADDED to the evaluation's running sums acc [3 T] (fp64, device): acc[t] +=
 * recall@topk[t] (rows whose first hit is < topk[t]), acc[T + t] += mrr@topk[t], acc[2 T + t] += the
 * batch's ndcg@topk[t] ratio.  topk [T] int32 on the device; B <= 4096, k <= 2048, T <= 16.          */
int drt_hit_metrics_i8(const int8_t* hit, int64_t B, int64_t k, const int32_t* topk, int32_t T, double* acc,
                       void* stream);

/* Merge `nparts` per-shard top-k lists into one global top-k.
 * scores/ids: [nparts, nq, k_in] (each part sorted score desc, id asc, as
 * drt_ip_topk_bf16 writes them); out: [nq, k_out], k_out <= k_in*nparts,
 * k_in <= 2048, nparts <= 64.                                                */
int drt_topk_merge(const float* scores, const int64_t* ids, int64_t nq, int32_t nparts,
                   int32_t k_in, int32_t k_out, float* out_scores, int64_t* out_ids,
                   void* stream);

/* ------------------------------------------------------------------------
 * Distributed exact top-k with ONE global threshold (row shards, one process
 * per GPU).  Replaces the same boundary as drt_ip_topk_bf16 + drt_topk_merge
 * (faiss search per partition + merge_retrieval_results_by_score,
 * DRT/evaluator/index.py:31-33, DRT/model/utils.py:215-229) with a protocol
 * that makes every shard filter against the threshold of the WHOLE corpus,
 * so each shard collects ~1/world of the candidates:
 *   1. drt_ip_topk_dist_sample   per shard: best r sampled keys  [nq][r] u32
 *   2. caller all-gathers the lists -> [world][nq][r]  (r = sample_rank(k))
 *   3. drt_ip_topk_dist_tau      tau[q] = r-th best over all lists
 *   4. drt_ip_topk_dist_filter   per shard: packed top-k [nq][k + 1] u64
 *        entry j < k: (desc score key << 32) | global id  (ascending = score
 *        desc, id asc; ~0 = empty), entry k: (valid entries << 32) | flags
 *        (bit 0 = shard overflow)
 *   5. caller all-gathers packed -> [world][nq][k + 1]
 *   6. drt_topk_merge_packed     exact merged top-k + status[q] (1 = not
 *        certified: fall back to the per-shard exact path for that batch)
 * Requires n_global < 2^32 (ids travel in 32 bits).                         */
int32_t drt_ip_topk_sample_rank(int32_t k);
size_t drt_ip_topk_dist_workspace(int64_t nq, int64_t n_local, int64_t n_global, int32_t d,
                                  int32_t k);
int drt_ip_topk_dist_sample(const void* Q, int64_t nq, const void* P, int64_t n_local,
                            int64_t n_global, int32_t d, int32_t k, uint32_t* best, void* ws,
                            size_t ws_bytes, void* stream);
int drt_ip_topk_dist_tau(const uint32_t* lists, int64_t nq, int32_t nlists, int32_t k, float* tau,
                         void* stream);
int drt_ip_topk_dist_filter(const void* Q, int64_t nq, const void* P, int64_t n_local,
                            int64_t n_global, int32_t d, int32_t k, int64_t id_offset,
                            const float* tau, uint64_t* packed, void* ws, size_t ws_bytes,
                            void* stream);
/* 4 over a shard in row chunks (d <= 768, n_local < 2^32): chunk c = rows [starts[c], starts[c + 1])
 * (host array of nchunks + 1 entries, starts[0] = 0, starts[nchunks] = n_local) is one filter scan
 * launch, all chunks append to one hit list and one select emits this shard's packed top-k -- the
 * same lists as drt_ip_topk_dist_filter over the whole shard (workspace: drt_ip_topk_dist_workspace
 * for n_local).  A group of query batches keeps its query blocks in step over each chunk. */
int drt_ip_topk_dist_filter_chunks(const void* Q, int64_t nq, const void* P, int64_t n_local,
                                   int64_t n_global, int32_t d, int32_t k, int64_t id_offset,
                                   const float* tau, uint64_t* packed, const int64_t* starts,
                                   int32_t nchunks, void* ws, size_t ws_bytes, void* stream);
/* 3+4 fused: tau from the gathered lists [nlists][nq][r] (written to tau_out when it is not
 * NULL) and this shard's packed top-k, with the hit counters zeroed by the threshold kernel
 * (3 launches).  Same results as drt_ip_topk_dist_tau followed by drt_ip_topk_dist_filter. */
int drt_ip_topk_dist_filter_lists(const void* Q, int64_t nq, const void* P, int64_t n_local,
                                  int64_t n_global, int32_t d, int32_t k, int64_t id_offset,
                                  const uint32_t* lists, int32_t nlists, float* tau_out,
                                  uint64_t* packed, void* ws, size_t ws_bytes, void* stream);
/* The same for query rows [q0, q0 + nq) of lists gathered for a larger query set (the batched
 * sample phase of a group of query batches): list j of this batch starts at
 * lists + j * lists_stride (u32 elements; lists_stride >= nq * r unless nlists == 1). */
int drt_ip_topk_dist_filter_lists_at(const void* Q, int64_t nq, const void* P, int64_t n_local,
                                     int64_t n_global, int32_t d, int32_t k, int64_t id_offset,
                                     const uint32_t* lists, int32_t nlists, int64_t lists_stride,
                                     float* tau_out, uint64_t* packed, void* ws, size_t ws_bytes,
                                     void* stream);
int drt_topk_merge_packed(const uint64_t* parts, int64_t nq, int32_t nparts, int32_t k,
                          int64_t n_global, float* out_scores, int64_t* out_ids, int32_t* status,
                          void* stream);
/* The same merge of lists of k entries certified at k_cert <= k (status 1 when fewer than k_cert
 * candidates exist overall or a shard overflowed): the canonical-order stage merges
 * drt_refine_width(k_cert) entries per shard.                                                  */
/* Capped exchange lists (round 6): parts [nparts][nq][lcap + 1], lcap <= k, each a shard's best lcap
 * packed keys (entry lcap = count << 32 | bit 0 overflow | bit 1 truncated: the shard had more hits than
 * it carries), merged into the top k with the certificate of drt_topk_merge_packed_cert plus: a truncated
 * list whose last entry ranks above the k-th merged place leaves its query uncertified (status 1).
 * 2 <= nparts <= 8, nparts * lcap <= 16384.  What a W-rank exchange carries instead of k + 1 entries.   */
int drt_topk_merge_packed_capped(const uint64_t* parts, int64_t nq, int32_t nparts, int32_t lcap, int32_t k,
                                 int32_t k_cert, int64_t n_global, float* out_scores, int64_t* out_ids,
                                 int32_t* status, void* stream);
int drt_topk_merge_packed_cert(const uint64_t* parts, int64_t nq, int32_t nparts, int32_t k,
                               int32_t k_cert, int64_t n_global, float* out_scores, int64_t* out_ids,
                               int32_t* status, void* stream);
/* Dense score matrix C[m, n] = A[m, d] . B[n, d]^T with fp32 accumulation
 * (torch.matmul(q_reps, p_reps.T), biencoder.py:107).  A, B bf16; C fp32 with
 * leading dimension ldc.                                                     */
int drt_gemm_nt_bf16_f32(const void* A, const void* B, float* C, int64_t m, int64_t n,
                         int32_t d, int64_t ldc, void* stream);

/* ------------------------------------------------------------------------
 * Bi-encoder forward building blocks (DRModel.encode, biencoder.py:127-151,
 * over HF BertModel; BERT post-LN layer = linear(QKV) -> attention ->
 * linear(out, +bias +residual, fp32) -> layernorm -> linear(FFN1, GELU) ->
 * linear(FFN2, +bias +residual, fp32) -> layernorm).
 * ------------------------------------------------------------------------
 * drt_embed_ln: out[B*L, H] bf16 = LN(word_emb[ids] + type_emb[type_ids or 0]
 *   + pos_emb[l]) (modeling_bert.py:53-107); tables/LN params fp32, H % 256 == 0.
 * drt_linear_bf16: Y = X . W^T (+bias)(GELU)(+residual); X [M,K], W [N,K] bf16,
 *   bias fp32 [N] or NULL, residual bf16 [M,N] or NULL; flags bit0 = GELU(erf),
 *   bit1 = fp32 output (else bf16).  K % 64 == 0.
 * drt_layernorm_f32_bf16: out bf16 = LN(X fp32 [M,H]).
 * drt_layernorm_bf16: out bf16 = LN(X bf16 [M,H]) (fp32 statistics); the
 *   encoder's default, fed by a bf16 +bias +residual epilogue (one rounding).
 * drt_attention_bf16: ctx[B*L, heads*64] = softmax(Q K^T * scale + mask) V per
 *   head, from packed qkv [B*L, 3*heads*64]; mask int64 [B,L] (1 token, 0 pad)
 *   or NULL; L <= 512, head_dim == 64.
 * drt_pool_bf16: reps fp32 [B,H] (+ optional bf16 copy) from hidden bf16
 *   [B,L,H]; mode 0 first, 1 masked mean, 2 max(hidden*mask) (utils.py:233-240).
 * drt_l2_normalize_f32: in place x /= max(||x||_2, 1e-12) per row.          */
int drt_embed_ln(const int64_t* ids, const int64_t* type_ids, int64_t B, int64_t L,
                 const float* word_emb, const float* pos_emb, const float* type_emb,
                 const float* gamma, const float* beta, float eps, int32_t H, void* out,
                 void* stream);
int drt_linear_bf16(const void* X, const void* W, const float* bias, const void* residual,
                    void* Y, int64_t M, int64_t N, int64_t K, int32_t flags, void* stream);
/* drt_linear_bf16_ws: the same with a caller workspace; shapes too small to fill the chip
 * (query-sized batches: < 384 tiles of 128^2, partials <= 16 MiB) split K over ~2 blocks
 * per CU into ws (fp32 partials) and finish with one fixed-order reduction + epilogue
 * (deterministic).
 * drt_linear_workspace(M, N, K) = the bytes it needs (0: no split for this shape).      */
size_t drt_linear_workspace(int64_t M, int64_t N, int64_t K);
int drt_linear_bf16_ws(const void* X, const void* W, const float* bias, const void* residual,
                       void* Y, int64_t M, int64_t N, int64_t K, int32_t flags, void* ws,
                       size_t ws_bytes, void* stream);
/* BertSelfOutput / BertOutput (modeling_bert.py:282-352: dense + residual + LayerNorm):
 * out = LayerNorm(bf16(X W^T + bias + residual)) * gamma + beta.  With a split-K plan (query-sized
 * batches, ws_bytes >= drt_linear_workspace) the partials are finished by ONE fused split-K +
 * LayerNorm launch; otherwise the bf16 pre-LayerNorm sum goes to `presum` [M, N] and is normalised.
 * Bit-identical to drt_linear_bf16_ws + drt_layernorm_bf16.  out may alias residual; N % 256 == 0,
 * N <= 1024.                                                                                       */
int drt_linear_ln_bf16_ws(const void* X, const void* W, const float* bias, const void* residual,
                          const float* gamma, const float* beta, float eps, void* presum, void* out,
                          int64_t M, int64_t N, int64_t K, void* ws, size_t ws_bytes, void* stream);
/* drt_linear_bf16_ws plus the training tower's epilogue fusions (bf16 Y):
 *   gelu_pre [M, N] != NULL: Y = (X W^T) * GELU'(gelu_pre)  (dgrad through an erf GELU whose input
 *     was gelu_pre; bias / residual / GELU / Y_pre / DROP must be off);
 *   Y_pre [M, N] != NULL (requires flags GELU): Y_pre = X W^T + b and Y = GELU(Y_pre);
 *   flags & 4 (DROP): Y = dropout(X W^T + b) + residual, the mask of drt_dropout_add_bf16 for
 *     (drop_p, seed, site) at the flat index m * N + n.
 * Replaces linear -> drt_gelu_bf16, dgrad -> drt_gelu_bwd_bf16 and linear -> drt_dropout_add_bf16
 * pairs of the training tower (BertIntermediate / BertOutput / BertSelfOutput under autograd). */
/* drt_linear_dgelu_bias_bf16: the FFN1 dgrad with its GELU backward and bias gradient:
 *   dX [M,N] bf16 = (dY[M,K] . Wt[N,K]^T) * GELU'(pre[M,N]) (as drt_linear_bf16_ex with gelu_pre),
 *   dbias [N] fp32 = column sums of the stored dX -- from the GEMM epilogue when the whole-line
 *   plan applies with N % 256 == 0 (no pass over dX), else summed after it.  ws of
 *   drt_linear_dgelu_bias_workspace(M, N, K) bytes.  (BertIntermediate, modeling_bert.py:325-337.) */
size_t drt_linear_dgelu_bias_workspace(int64_t M, int64_t N, int64_t K);
int drt_linear_dgelu_bias_bf16(const void* dY, const void* Wt, const void* gelu_pre, void* dX, int64_t M,
                               int64_t N, int64_t K, float* dbias, void* ws, size_t ws_bytes, void* stream);
int drt_linear_bf16_ex(const void* X, const void* W, const float* bias, const void* residual,
                       const void* gelu_pre, void* Y, void* Y_pre, int64_t M, int64_t N, int64_t K,
                       int32_t flags, float drop_p, uint64_t seed, uint64_t site, void* ws,
                       size_t ws_bytes, void* stream);
int drt_layernorm_f32_bf16(const float* X, int64_t M, int32_t H, const float* gamma,
                           const float* beta, float eps, void* out, void* stream);
int drt_layernorm_bf16(const void* X, int64_t M, int32_t H, const float* gamma,
                       const float* beta, float eps, void* out, void* stream);
int drt_attention_bf16(const void* qkv, const int64_t* mask, void* ctx, int64_t B, int64_t L,
                       int32_t heads, int32_t head_dim, float scale, void* stream);
/* drt_attention_fwd_lse_bf16: the same forward, also writing lse [B][heads][L] fp32 = the
 * log-sum-exp of each query's scaled, masked scores (input of the attention backward).  */
int drt_attention_fwd_lse_bf16(const void* qkv, const int64_t* mask, void* ctx, float* lse, int64_t B,
                               int64_t L, int32_t heads, int32_t head_dim, float scale, void* stream);

/* ------------------------------------------------------------------------
 * Encoder backward building blocks (the gradient of HF BertModel's
 * ops as the training step of run_random_sampling.py takes it under autograd,
 * DRT/trainer/trainer.py:113-133; transformers modeling_bert.py:282-352).
 * ------------------------------------------------------------------------
 * drt_layernorm_bwd_bf16: dx [M,H] bf16 = LN backward of dy through LN(x) with gamma (x = the
 *   bf16 pre-LN sums the forward stored; statistics recomputed) + dres (residual gradient or
 *   NULL); dgamma / dbeta fp32 [H], deterministic (fixed-order partial sums in ws of
 *   drt_layernorm_bwd_workspace(M, H) bytes).  H % 256 == 0, H <= 1024.
 * drt_colsum_bf16: out[n] fp32 = sum_rows x[row][n] (bias gradients), fixed order, ws of
 *   drt_colsum_workspace(M, N) bytes (0 for M < 256).
 * drt_gelu_bwd_bf16: dx = dy * (Phi(x) + x phi(x)) for the erf GELU (pre = the FFN1
 *   pre-activation), n elements.
 * drt_transpose_bf16: y [C,R] = x [R,C]^T (operand layout for the weight gradients).      */
size_t drt_layernorm_bwd_workspace(int64_t M, int32_t H);
int drt_layernorm_bwd_bf16(const void* dy, const void* x, const float* gamma, float eps, int64_t M,
                           int32_t H, const void* dres, void* dx, float* dgamma, float* dbeta,
                           void* ws, size_t ws_bytes, void* stream);
/* The same, also writing dx_drop = dropout(dx) with drt_dropout_add_bf16's mask of
 * (drop_p, seed, site) at the flat index m * H + h (the gradient of a linear whose output was
 * dropped before this LayerNorm's residual add; replaces a separate dropout pass).          */
int drt_layernorm_bwd_drop_bf16(const void* dy, const void* x, const float* gamma, float eps,
                                int64_t M, int32_t H, const void* dres, void* dx, void* dx_drop,
                                float drop_p, uint64_t seed, uint64_t site, float* dgamma,
                                float* dbeta, void* ws, size_t ws_bytes, void* stream);
/* The same, also writing dsum [H] fp32 = the column sums of the gradient it hands down (dx_drop,
 * or dx when dx_drop is NULL): the bias gradient of the linear feeding this LayerNorm
 * (BertSelfOutput / BertOutput dense.bias) without a separate pass over that gradient.   */
int drt_layernorm_bwd_sum_bf16(const void* dy, const void* x, const float* gamma, float eps,
                               int64_t M, int32_t H, const void* dres, void* dx, void* dx_drop,
                               float drop_p, uint64_t seed, uint64_t site, float* dgamma,
                               float* dbeta, float* dsum, void* ws, size_t ws_bytes, void* stream);
size_t drt_colsum_workspace(int64_t M, int64_t N);
int drt_colsum_bf16(const void* x, int64_t M, int64_t N, float* out, void* ws, size_t ws_bytes,
                    void* stream);
/* drt_colsum_f32: the same over an fp32 matrix (partial sums of the fused bias gradients).  */
int drt_colsum_f32(const float* x, int64_t M, int64_t N, float* out, void* ws, size_t ws_bytes,
                   void* stream);
int drt_gelu_bwd_bf16(const void* dy, const void* pre, int64_t n, void* dx, void* stream);
int drt_transpose_bf16(const void* x, int64_t R, int64_t C, void* y, void* stream);
/* drt_transpose_bf16_ld: the same into y with row stride ldy >= R (padded GEMM operands). */
int drt_transpose_bf16_ld(const void* x, int64_t R, int64_t C, void* y, int64_t ldy, void* stream);
/* drt_linear_wgrad_bf16: dW [N,K] fp32 = dY[T,N]^T . X[T,K] (nn.Linear weight gradient) straight
 *   from the token-major operands (no transposed copies): T % 32 == 0, N % 8 == 0, K % 8 == 0;
 *   ws of drt_linear_wgrad_workspace(T, N, K) bytes (deterministic split over T; 0 = none).  */
size_t drt_linear_wgrad_workspace(int64_t T, int64_t N, int64_t K);
int drt_linear_wgrad_bf16(const void* dY, const void* X, float* dW, int64_t T, int64_t N, int64_t K, void* ws,
                          size_t ws_bytes, void* stream);
/* drt_attention_bwd_bf16: dqkv [B*L, 3H] (dQ | dK | dV in qkv's packed layout) of the
 * attention forward, from qkv, its ctx = O, dctx = dO, the forward's lse and the key mask;
 * L <= 512, head_dim 64 (BertSelfAttention under autograd, modeling_bert.py:164-204);
 * L <= 160: one work-group per (sequence, head) holding the sequence in LDS; 160 < L <= 512:
 * streamed dK/dV and dQ kernels over 128-row groups (dropout there needs the forward's bits). */
/* drt_embed_ln_pre: drt_embed_ln that also writes the bf16 pre-LN sum (word + type + pos).
 * drt_gelu_bf16: y = GELU(x) elementwise (erf form).
 * drt_embedding_bwd: scatter-add of d [B*L, H] (gradient of the pre-LN embedding sum) into
 *   dword [V,H], dpos [P,H], dtype [types,H] fp32 (caller zeroes them: word rows by atomics,
 *   position rows by chunked column sums, token type 0 from the position sums when
 *   type_ids is NULL); tokens equal to padding_idx (nn.Embedding(padding_idx), -1 = none)
 *   add nothing to dword.                                                                   */
int drt_embed_ln_pre(const int64_t* ids, const int64_t* type_ids, int64_t B, int64_t L,
                     const float* word_emb, const float* pos_emb, const float* type_emb,
                     const float* gamma, const float* beta, float eps, int32_t H, void* out, void* pre,
                     void* stream);
int drt_gelu_bf16(const void* x, int64_t n, void* y, void* stream);
int drt_embedding_bwd(const int64_t* ids, const int64_t* type_ids, const void* d, int64_t B, int64_t L,
                      int32_t H, int64_t padding_idx, float* dword, float* dpos, float* dtype,
                      void* stream);
/* drt_embedding_bwd with the token-type table's row count (type_vocab_size <= 4 when type_ids is
 * given; BERT: 2): the type rows' gradients are per-type column sums over token chunks (drt_embedding_bwd
 * assumes 2 rows).                                                                            */
int drt_embedding_bwd_types(const int64_t* ids, const int64_t* type_ids, int32_t ntypes, const void* d,
                            int64_t B, int64_t L, int32_t H, int64_t padding_idx, float* dword, float* dpos,
                            float* dtype, void* stream);
int drt_attention_bwd_bf16(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                           const int64_t* mask, void* dqkv, int64_t B, int64_t L, int32_t heads,
                           int32_t head_dim, float scale, void* stream);
/* Training dropout (HF train mode, modeling_bert.py:107,195,296,348): keep element i of a
 * site iff drop_hash24(seed, site, i) >= p 2^24 (csrc/drt_common.h), kept values / (1 - p).
 * drt_attention_train_fwd_bf16 / _bwd_bf16: attention with dropout of the probabilities
 *   (element index ((b*heads + head)*L + q)*L + key); p = 0 is the plain forward / backward.
 * drt_dropout_add_bf16: out = dropout(y) + resid (resid may be NULL) over n elements; the
 *   same call on a gradient with resid = NULL is the dropout backward.                      */
int drt_attention_train_fwd_bf16(const void* qkv, const int64_t* mask, void* ctx, float* lse, int64_t B,
                                 int64_t L, int32_t heads, int32_t head_dim, float scale, float drop_p,
                                 uint64_t seed, uint64_t site, void* stream);
int drt_attention_train_bwd_bf16(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                                 const int64_t* mask, void* dqkv, int64_t B, int64_t L, int32_t heads,
                                 int32_t head_dim, float scale, float drop_p, uint64_t seed, uint64_t site,
                                 void* stream);
int drt_dropout_add_bf16(const void* y, const void* resid, int64_t n, float p, uint64_t seed, uint64_t site,
                         void* out, void* stream);
/* The training attention pair with the dropout keep mask kept as bits: the forward writes
 * drop_bits [B][heads][L][ceil(L / 32)] u32 (bit key & 31 of word (query, key >> 5); only when
 * drop_p > 0 and drop_bits != NULL), the backward reads them instead of regenerating the hash
 * twice per (query, key).  Same masks, same results as the hash-regenerating pair.  For
 * L > 160 with drop_p > 0 the backward requires drop_bits (DRT_EINVAL without).              */
int drt_attention_train_fwd_bits_bf16(const void* qkv, const int64_t* mask, void* ctx, float* lse,
                                      uint32_t* drop_bits, int64_t B, int64_t L, int32_t heads,
                                      int32_t head_dim, float scale, float drop_p, uint64_t seed,
                                      uint64_t site, void* stream);
int drt_attention_train_bwd_bits_bf16(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                                      const int64_t* mask, const uint32_t* drop_bits, void* dqkv, int64_t B,
                                      int64_t L, int32_t heads, int32_t head_dim, float scale, float drop_p,
                                      uint64_t seed, uint64_t site, void* stream);
/* drt_attention_train_bwd_bias_bf16: the same, also writing dbias [3H] fp32 = the column sums of
 * dQKV (the query / key / value bias gradients of BertSelfAttention) from per-sequence (L > 160:
 * per 128-row group) partials left in ws (drt_attention_train_bwd_bias_workspace bytes, sized for
 * any L <= 512), reduced in a fixed order, without a pass over dQKV.                          */
size_t drt_attention_train_bwd_bias_workspace(int64_t B, int32_t heads, int32_t head_dim);
int drt_attention_train_bwd_bias_bf16(const void* qkv, const void* ctx, const void* dctx, const float* lse,
                                      const int64_t* mask, const uint32_t* drop_bits, void* dqkv, int64_t B,
                                      int64_t L, int32_t heads, int32_t head_dim, float scale, float drop_p,
                                      uint64_t seed, uint64_t site, float* dbias, void* ws, size_t ws_bytes,
                                      void* stream);
int drt_pool_bf16(const void* hidden, const int64_t* mask, int64_t B, int64_t L, int32_t H,
                  int32_t mode, float* out, void* out_bf16, void* stream);
int drt_l2_normalize_f32(float* x, int64_t B, int32_t H, void* out_bf16, void* stream);
/* ------------------------------------------------------------------------
 * In-batch-negative training loss (DRModel.forward, biencoder.py:107-119;
 * SimpleContrastiveLoss, losses.py:11-17), fp32 like the reference.
 * ------------------------------------------------------------------------
 * drt_gemm_nt_f32: C[m,n] = A[m,k] . B[n,k]^T on the exact-f32 MFMA.
 * drt_ce_fwd: per row lse_i = log sum_j exp(S_ij), row_loss_i = lse_i - S_i,t
 *   with t = i * target_stride; *loss = scale * mean_i row_loss_i
 *   (deterministic order).  All device pointers.
 * drt_ce_bwd: dS_ij = grad * scale / m * (softmax(S)_ij - [j == t]); grad is
 *   a device scalar (NULL = 1).
 * drt_transpose_f32: Y[cols, rows] = X[rows, cols]^T.                       */
int drt_gemm_nt_f32(const float* A, const float* B, float* C, int64_t m, int64_t n, int64_t k,
                    int64_t lda, int64_t ldb, int64_t ldc, void* stream);
/* drt_gemm_f32: C[m,n] = sum_k A(m,k) B(k,n), exact-f32 MFMA, for the score matrix and its
 * backward without transposes (replaces torch.matmul in DRModel.forward, biencoder.py:107, and
 * the autograd of it).  a_kc: A stored [m][lda>=k] (else [k][lda>=m]); b_kc: B stored
 * [n][ldb>=k] (else [k][ldb>=n]).  splits > 1: deterministic split-K through ws
 * (splits * m * n floats, partial sums added in a fixed order).                        */
int drt_gemm_f32(const float* A, const float* B, float* C, int64_t m, int64_t n, int64_t k, int64_t lda,
                 int64_t ldb, int64_t ldc, int32_t a_kc, int32_t b_kc, int32_t splits, float* ws, void* stream);
int drt_ce_fwd(const float* S, int64_t m, int64_t n, int64_t target_stride, float scale,
               float* lse, float* row_loss, float* loss, void* stream);
int drt_ce_bwd(const float* S, const float* lse, int64_t m, int64_t n, int64_t target_stride,
               const float* grad, float scale, float* dS, void* stream);
int drt_transpose_f32(const float* X, int64_t rows, int64_t cols, float* Y, void* stream);
/* Fused score + CE, one host call per direction (the path score_ce.ScoreCE uses;
 * replaces the matmul + CrossEntropyLoss of DRModel.forward, biencoder.py:107-119,
 * and their autograd).  q [m,d], p [n,d] fp32 row-major; target t_i = i * target_stride.
 * drt_score_ce_fwd: S [m,n], lse [m], *loss (3 launches: split-K GEMM, per-row split
 *   reduction + LSE + row loss, fixed-order mean).
 * drt_score_ce_bwd: dq [m,d] = dS . p, dp [n,d] = dS^T . q with dS as drt_ce_bwd
 *   (3 launches: dS, both GEMMs in one grid, both fixed-order split reductions).
 * Both need ws of drt_score_ce_workspace(m, n, d) bytes (scratch only; results are
 * bit-identical to drt_gemm_f32 + drt_ce_fwd / drt_ce_bwd).                  */
size_t drt_score_ce_workspace(int64_t m, int64_t n, int32_t d);
int drt_score_ce_fwd(const float* q, const float* p, int64_t m, int64_t n, int32_t d, int64_t target_stride,
                     float scale, float* S, float* lse, float* loss, void* ws, size_t ws_bytes, void* stream);
int drt_score_ce_bwd(const float* q, const float* p, const float* S, const float* lse, int64_t m, int64_t n,
                     int32_t d, int64_t target_stride, const float* grad, float scale, float* dq, float* dp,
                     void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Launch timing (measurement support for bench.py's roofline figure).
 * When enabled, every launch of the named kernel family is bracketed by a
 * pair of hipEvents recorded on the stream it is launched on.
 * family: 0 = ip_scan FILTER pass (the HBM-bound search kernel),
 *         1 = ip_scan sample pass, 2 = select, 3 = merge, 4 = gemm.
 * drt_profile_read synchronises on the recorded events and returns the sum of
 * their durations (ms) and the launch count, then clears the record.        */
int drt_profile_enable(int32_t family, int32_t enable);
int drt_profile_read(int32_t family, double* total_ms, int64_t* count);
/* The same, launch by launch: the first min(cap, recorded) durations (ms) in launch order go to
 * ms_each, *count = the number recorded; the record is cleared.                                 */
int drt_profile_read_each(int32_t family, double* ms_each, int64_t cap, int64_t* count);

#ifdef __cplusplus
}
#endif

#endif /* DRT_H_ */
