#!/usr/bin/env python3
"""Canonical-order stage probe (round 6): a 2048-query group over the 10M x 768 bench corpus through the
one-GPU grouped path's candidate lists (sample -> tau -> chunked filter -> merge), then `--reps` timed
launches of the local refine_delta (prep + exact sums of the window's candidates) and one refine_sort.
Prints the time per call and an order-independent digest of the deltas (variants must match).
usage: python tools/refine_probe.py [--n 10000000] [--reps 10]   (DRT_LIB=<variant .so> for an A/B)"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--queries", type=int, default=2048)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch
    from bench import gen_shard
    from denseretrievaltoolkits_amd import kernels, ops
    from denseretrievaltoolkits_amd import search as srch
    dev = torch.device("cuda", 0)
    p, _, _ = gen_shard(a.n, 1, 0, 768, dev)
    g = torch.Generator(device=dev).manual_seed(5678)
    q = torch.randn((a.queries, 768), generator=g, device=dev).to(torch.bfloat16)
    k = a.k
    kc = kernels.refine_width(k)
    stats = kernels.row_stats(p)
    tau = kernels.dist_tau(kernels.dist_sample(q, p, a.n, k)[None].contiguous(), k)
    chunks = srch.group_chunks(a.n)
    packed = torch.empty((a.queries, kc + 1), dtype=torch.int64, device=dev)
    kernels.dist_filter_chunks_into(q, p, a.n, kc, 0, tau, [c for c, _ in chunks] + [chunks[-1][1]], packed)
    s, i, st = kernels.merge_packed(packed[None], kc, a.n, k_cert=k)
    drt = ops.load()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        delta, cnt = drt.refine_delta(q, p, 0, s, i, k, stats, tau, st.clone(), True)
    e0.record()
    for _ in range(a.reps):
        delta, cnt = drt.refine_delta(q, p, 0, s, i, k, stats, tau, st.clone(), True)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    win = cnt[:, 0].clamp_min(0).double()
    inwin = torch.arange(delta.shape[1], device=dev)[None, :] < cnt[:, :1]   # only the window is written
    dv = torch.where(inwin, delta.double(), torch.zeros((), dtype=torch.float64, device=dev))
    dig = float((dv * torch.arange(1, delta.numel() + 1, device=dev, dtype=torch.float64)
                 .remainder(997).view_as(delta)).sum().item())
    print(json.dumps({"queries": a.queries, "rows": a.n, "refine_delta_ms": round(ms, 4),
                      "window_mean": round(float(win.mean()), 1),
                      "gathered_GB": round(float(win.sum()) * 768 * 2 / 1e9, 3),
                      "GBps": round(float(win.sum()) * 768 * 2 / (ms * 1e-3) / 1e9, 1), "digest": dig}), flush=True)


if __name__ == "__main__":
    main()
