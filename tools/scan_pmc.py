#!/usr/bin/env python3
"""Filter-scan launches for PMC passes: the 10M x 768 shard, 128 Gaussian queries, three launches of
drt_ip_topk_dist_filter per threshold -- no hits (tau = +inf), exactly 4096 hits per query (the
rank-4096 score, dense fp32 torch reference), and the product's own sampled tau (what ip_topk's filter
pass runs against: ~4k hits per query with the sample's spread).  Run under
`rocprofv3 --pmc ... -- python3 tools/scan_pmc.py`; the filter dispatches come in that order, three
each (tools/pmc_report.py-style grouping by dispatch order).
usage: python tools/scan_pmc.py [--n 10000000]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--k", type=int, default=1000)
    a = ap.parse_args()
    import torch
    from bench import gen_shard
    from denseretrievaltoolkits_amd import kernels
    dev = torch.device("cuda", 0)
    p, _, _ = gen_shard(a.n, 1, 0, 768, dev)
    g = torch.Generator(device=dev).manual_seed(5678)
    q = torch.randn((128, 768), generator=g, device=dev).to(torch.bfloat16)
    taus = [torch.full((128,), float("inf"), device=dev)]
    taus.append(torch.cat([(q.float() @ p[s: s + 2_000_000].float().T) for s in range(0, a.n, 2_000_000)],
                          1).topk(4096, dim=1).values[:, -1].contiguous())
    taus.append(kernels.dist_tau(kernels.dist_sample(q, p, a.n, a.k)[None].contiguous(), a.k))
    torch.cuda.synchronize()
    for tau in taus:
        for _ in range(3):
            kernels.dist_filter(q, p, a.n, a.k, 0, tau)
        torch.cuda.synchronize()
    print("scan_pmc: 3 thresholds x 3 filter launches", flush=True)


if __name__ == "__main__":
    main()
