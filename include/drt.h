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

/* Library version / self-description (host only, no GPU needed). */
const char* drt_version(void);

/* ------------------------------------------------------------------------
 * Brute-force inner-product top-k over one row shard  (index.py:16-33)
 * ------------------------------------------------------------------------
 * Q: [nq, d] bf16 queries.  P: [n, d] bf16 corpus shard (row i has global id
 * id_offset + i).  d must be a multiple of 64 and <= 1024; 1 <= k <= 2048.
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
 * drt_ip_topk_bf16) is non-zero.  SYNCHRONOUS: reads status back, allocates
 * scratch, rescans the shard for those queries only, and clears their status.
 * Returns the number of resolved queries in *n_resolved (may be NULL).      */
int drt_ip_topk_resolve(const void* Q, int64_t nq, const void* P, int64_t n, int32_t d,
                        int32_t k, int64_t id_offset, float* out_scores, int64_t* out_ids,
                        int32_t* status, int64_t* n_resolved, void* stream);

/* Merge `nparts` per-shard top-k lists into one global top-k.
 * scores/ids: [nparts, nq, k_in] (each part sorted score desc, id asc, as
 * drt_ip_topk_bf16 writes them); out: [nq, k_out], k_out <= k_in*nparts,
 * k_in <= 2048, nparts <= 64.                                                */
int drt_topk_merge(const float* scores, const int64_t* ids, int64_t nq, int32_t nparts,
                   int32_t k_in, int32_t k_out, float* out_scores, int64_t* out_ids,
                   void* stream);

/* Dense score matrix C[m, n] = A[m, d] . B[n, d]^T with fp32 accumulation
 * (torch.matmul(q_reps, p_reps.T), biencoder.py:107).  A, B bf16; C fp32 with
 * leading dimension ldc.                                                     */
int drt_gemm_nt_bf16_f32(const void* A, const void* B, float* C, int64_t m, int64_t n,
                         int32_t d, int64_t ldc, void* stream);

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

#ifdef __cplusplus
}
#endif

#endif /* DRT_H_ */
