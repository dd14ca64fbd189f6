#!/usr/bin/env python3
"""Filter-scan probe: time ONE filter launch (drt_ip_topk_dist_filter: filter scan + select) over an
n-row bf16 shard for 128 Gaussian queries, against thresholds that admit a chosen number of hits
per query (the scores' rank-R value; R = 0 means no hits), in both hit-append flavours (picked by
the expected-hit estimate the call derives from n_global).  HIP events on torch's stream.
usage: python tools/scan_probe.py [--n 1000000] [--reps 20] [--ranks 0,1000,2000] (-1: the sampled tau)"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ranks", default="0,1000,2000")
    ap.add_argument("--k", type=int, default=1000)
    args = ap.parse_args()
    import torch
    from bench import gen_shard
    from denseretrievaltoolkits_amd import kernels
    dev = torch.device("cuda", 0)
    p, _, _ = gen_shard(args.n, 1, 0, 768, dev)
    g = torch.Generator(device=dev).manual_seed(5678)
    q = torch.randn((128, 768), generator=g, device=dev).to(torch.bfloat16)
    ranks = [int(x) for x in args.ranks.split(",")]
    # tau of rank R = the R-th best exact score (the product's own certified top-R, R <= 2048)
    taus = {}
    for R in ranks:
        if R == 0:
            taus[R] = torch.full((128,), float("inf"), device=dev)
        elif R < 0:   # the product's own sampled threshold (what ip_topk's filter pass runs against)
            taus[R] = kernels.dist_tau(kernels.dist_sample(q, p, args.n, args.k)[None].contiguous(), args.k)
        elif R <= 2048:
            sc, _, _ = kernels.ip_topk(q, p, R)
            taus[R] = sc[:, R - 1].contiguous()
        else:   # past the kernel's k bound: a dense fp32 torch reference (rank-R score, near-exact)
            taus[R] = torch.cat([(q.float() @ p[a: a + 2_000_000].float().T) for a in range(0, p.shape[0], 2_000_000)],
                                1).topk(R, dim=1).values[:, R - 1].contiguous()
    torch.cuda.synchronize()
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()

    def prof_read(fam):
        tot, cnt = _native.ctypes.c_double(0.0), _native.c_i64(0)
        lib.drt_profile_read(fam, _native.ctypes.byref(tot), _native.ctypes.byref(cnt))
        return tot.value / max(1, cnt.value) * 1e3
    out = {}
    # the product's one-GPU call (sample -> threshold -> filter -> select) for comparison
    for _ in range(2):
        kernels.ip_topk(q, p, args.k, resolve=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for fam in (0, 1, 2):
        lib.drt_profile_enable(fam, 1)
    e0.record()
    for _ in range(args.reps):
        kernels.ip_topk(q, p, args.k, resolve=False)
    e1.record()
    torch.cuda.synchronize()
    for fam in (0, 1, 2):
        lib.drt_profile_enable(fam, 0)
    out["ip_topk_us"] = round(e0.elapsed_time(e1) / args.reps * 1e3, 1)
    print(f"ip_topk (whole call): {out['ip_topk_us']} us: filter scan {prof_read(0):.1f}, sample scan "
          f"{prof_read(1):.1f}, select + threshold {prof_read(2):.1f} us per launch", flush=True)
    for R in ranks:
        tau = taus[R]
        if R < 0:
            hits = sum(((q.float() @ p[a: a + 2_000_000].float().T) >= tau[:, None]).sum(1)
                       for a in range(0, p.shape[0], 2_000_000)).float()
            print(f"sampled tau: hits/query mean {hits.mean().item():.0f} min {hits.min().item():.0f} "
                  f"max {hits.max().item():.0f}", flush=True)
        for flav, ng in (("dense", args.n), ("sparse", 10 * args.n)):
            for _ in range(2):
                kernels.dist_filter(q, p, ng, args.k, 0, tau)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            lib.drt_profile_enable(_native.PROF_SCAN, 1)
            lib.drt_profile_enable(2, 1)
            e0.record()
            for _ in range(args.reps):
                kernels.dist_filter(q, p, ng, args.k, 0, tau)
            e1.record()
            torch.cuda.synchronize()
            lib.drt_profile_enable(_native.PROF_SCAN, 0)
            lib.drt_profile_enable(2, 0)
            scan_us, sel_us = prof_read(_native.PROF_SCAN), prof_read(2)
            print(f"   scan {scan_us:.1f} us, select {sel_us:.1f} us", flush=True)
            us = e0.elapsed_time(e1) / args.reps * 1e3
            gbs = args.n * 768 * 2 / (us * 1e-6) / 1e9
            out[f"R{R}_{flav}"] = {"us": round(us, 1), "GBs": round(gbs, 0)}
            print(f"hits/query {R:6d} flavour {flav:6s}: {us:8.1f} us  {gbs:7.0f} GB/s (filter + select)", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
