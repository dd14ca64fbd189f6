#!/usr/bin/env python3
"""Grouped filter-scan launches for PMC passes: a 1.25M x 768 chunk (the W = 8 shard and the one-GPU
group chunk), 2048 Gaussian queries (16 query blocks), the product's sampled threshold; `--reps` launches
of drt_ip_topk_dist_filter_into exactly as search._gtau_enqueue_group issues them.  Run under
`rocprofv3 --pmc ... -- python3 tools/scan_group_pmc.py`; prints the launch time (HIP events).
usage: python tools/scan_group_pmc.py [--rows 1250000] [--queries 2048] [--reps 5]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_250_000)
    ap.add_argument("--queries", type=int, default=2048)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--hits", type=int, default=512,
                    help="hits per query the threshold admits in this chunk (512 = the product's ~4096 per query "
                         "over a 10M corpus; 0 = none)")
    a = ap.parse_args()
    import torch
    from bench import gen_shard
    from denseretrievaltoolkits_amd import kernels
    dev = torch.device("cuda", 0)
    p, _, _ = gen_shard(a.rows, 1, 0, 768, dev)
    g = torch.Generator(device=dev).manual_seed(5678)
    q = torch.randn((a.queries, 768), generator=g, device=dev).to(torch.bfloat16)
    n_global = a.rows * 8   # a chunk of a 10M corpus: ~1/8 of a query's ~4096 hits land in it
    if a.hits > 0:
        tau = torch.cat([(q[b:b + 256].float() @ p.float().T).topk(a.hits, dim=1).values[:, -1]
                         for b in range(0, a.queries, 256)]).contiguous()
    else:
        tau = torch.full((a.queries,), float("inf"), device=dev)
    kc = kernels.refine_width(a.k)
    packed = torch.empty((a.queries, kc + 1), dtype=torch.int64, device=dev)
    kernels.dist_filter_into(q, p, n_global, kc, 0, tau, packed)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        kernels.dist_filter_into(q, p, n_global, kc, 0, tau, packed)
    e1.record()
    torch.cuda.synchronize()
    hits = (packed[:, kc] >> 32).float()
    print(json.dumps({"rows": a.rows, "queries": a.queries, "ms_per_launch": round(e0.elapsed_time(e1) / a.reps, 4),
                      "valid_per_query_mean": round(float(hits.mean()), 1),
                      # order-independent digest of the packed lists (variants must match bit for bit)
                      "digest": int((packed.view(torch.int32).reshape(-1).double() * torch.arange(1, 2 * packed.numel() + 1,
                                     device=dev, dtype=torch.float64).remainder(1009)).sum().item())}), flush=True)


if __name__ == "__main__":
    main()
