"""Near-tie windows of the C2 leg's data (diagnostic for the canonical-order bound).

Encodes the C2 leg's corpus (random-init BERT-base, uniform token ids, 128-token passages, CLS
pooling: bench_legs.run_evaluate_c2) and a batch of 32-token queries on the HIP encoder, then per
query: the exact (fp64) scores of every row, the fp32 MFMA scores (drt_gemm_nt_bf16_f32), the worst
fp32 error in units of u * sum_i |q_i p_i|, and how many rows lie within 2 eps of the k-th exact score
for eps = c * u * ||q|| * max ||p|| at several c (c = 1920 is refine_eps's 2.5 d at d = 768).
Prints one JSON object.
"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def main(n=1_000_000, nq=256, k=1000, p_len=128, q_len=32, bs=512):
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd import kernels
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    lm = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(lm, dev)

    def encode(count, L, seed):
        out = torch.empty((count, 768), dtype=torch.bfloat16, device=dev)
        for j, a in enumerate(range(0, count, bs)):
            b = min(count, a + bs)
            rng = np.random.default_rng((seed, j))
            ids = rng.integers(1000, 30522, size=(b - a, L), dtype=np.int64)
            ids[:, 0], ids[:, -1] = 101, 102
            it = torch.from_numpy(ids).to(dev)
            m = torch.ones_like(it)
            h = enc(it, m)
            _, rb = enc.pool(h, m, "first", want_bf16=True)
            out[a:b] = rb
        return out

    t0 = time.time()
    P = encode(n, p_len, 11)
    Q = encode(nq, q_len, 12)
    torch.cuda.synchronize()
    res = {"n": n, "nq": nq, "k": k, "encode_s": round(time.time() - t0, 1)}
    u = 2.0 ** -24
    pn = P.double().pow(2).sum(1).sqrt()
    pmax = float(pn.max())
    res["p_norm_min_max"] = [float(pn.min()), pmax]
    qn = Q.double().pow(2).sum(1).sqrt()
    Pd = P.double()
    Pa = Pd.abs()
    windows = {c: [] for c in (1920, 400, 200, 100, 50, 25)}
    errs, scan_errs, gaps, spread, exact_ids = [], [], [], [], []
    for a in range(0, nq, 16):
        q = Q[a:a + 16]
        ex = q.double() @ Pd.T                       # [16, n] exact (fp64) scores
        f32 = kernels.gemm_nt_f32(q, P)                       # [16, n] MFMA fp32 scores
        ab = q.double().abs() @ Pa.T
        errs.append(float(((f32.double() - ex).abs() / (u * ab)).max()))
        s32, i32, _ = kernels.ip_topk(q, P, k)                # the filter scan's own fp32 scores
        exg = ex.gather(1, i32)
        scan_errs.append(float(((s32.double() - exg).abs() / (u * ab.gather(1, i32))).max()))
        exact_ids.append((-ex).sort(dim=1, stable=True).indices[:, :k])   # fp64 order, ties by ascending id
        srt = ex.sort(1, descending=True).values
        sk = srt[:, k - 1]
        spread.append((srt[:, 0] - srt[:, -1]).cpu().numpy() / (qn[a:a + 16] * pmax).cpu().numpy())
        gaps.append(((srt[:, k - 2] - srt[:, k]) / (qn[a:a + 16] * pmax)).cpu().numpy())
        for c in windows:
            eps = c * u * qn[a:a + 16] * pmax
            windows[c].append((srt >= (sk - 2 * eps)[:, None]).sum(1).cpu().numpy())
        del ex, f32, ab, srt
    res["max_fp32_err_over_u_abssum"] = max(errs)
    res["scan_topk_err_over_u_abssum"] = max(scan_errs)
    res["score_range_rel"] = float(np.concatenate(spread).max())
    res["kth_neighbour_gap_rel_median"] = float(np.median(np.concatenate(gaps)))
    res["window_rows"] = {str(c): {"median": int(np.median(np.concatenate(v))), "p90": int(np.percentile(np.concatenate(v), 90)),
                                   "max": int(np.concatenate(v).max())} for c, v in windows.items()}
    # the product index on the same data: canonical ids vs the fp64 order, certification counters
    from denseretrievaltoolkits_amd import search as srch
    ei = torch.cat(exact_ids)
    for name, gmin in (("per_batch", 1 << 62), ("grouped", 0)):
        srch.GROUP_MIN_ROWS, saved = gmin, srch.GROUP_MIN_ROWS
        idx = srch.FlatIPIndex.from_rows(P)
        torch.cuda.synchronize()
        t0 = time.time()
        out = idx.search_batches([Q[a:a + 128] for a in range(0, nq, 128)], k)
        torch.cuda.synchronize()
        dt = time.time() - t0
        srch.GROUP_MIN_ROWS = saved
        gi = torch.cat([o[1] for o in out])
        res["product_" + name] = {"ids_equal_frac": float((gi == ei).float().mean()),
                                  "queries_equal": int((gi == ei).all(1).sum()), "s": round(dt, 4),
                                  "order_uncertified": idx.order_uncertified, "wide_resolved": idx.wide_resolved,
                                  "resolved": idx.resolved}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    sys.exit(main(*[int(x) for x in sys.argv[1:]]))
