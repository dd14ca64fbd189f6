#!/usr/bin/env python3
"""Interleaved A/B of FlatIPIndex.search_batches paths on the bench workload (10M x 768 bf16,
Qb 128, k 1000), one process: grouped (search.GROUP_QUERIES per group) vs per-batch.
usage: python tools/search_ab.py [--rounds 3] [--steps 32] [--groups 2048,0]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--groups", default="2048,0")
    ap.add_argument("--order", choices=["exact", "fp32"], default="exact")
    args = ap.parse_args()
    import torch
    from bench import gen_shard
    from denseretrievaltoolkits_amd import search as srch
    dev = torch.device("cuda", 0)
    shard, _, _ = gen_shard(args.n, 1, 0, 768, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(5678)
    qs = torch.randn((args.steps, 128, 768), generator=g, device=dev).to(torch.bfloat16)
    srch.EXACT_ORDER = args.order == "exact"
    idx = srch.FlatIPIndex.from_rows(shard)
    batches = [qs[j] for j in range(args.steps)]
    variants = [int(v) for v in args.groups.split(",")]
    times = {v: [] for v in variants}
    ref = None
    for rnd in range(args.rounds):
        for v in variants:
            if v == 0:
                srch.GROUP_MIN_ROWS = 1 << 62
            else:
                srch.GROUP_MIN_ROWS = 0
                srch.GROUP_QUERIES = v
            idx.search_batches(batches[:2], 1000)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = idx.search_batches(batches, 1000)
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / args.steps * 1e3)
            ids = torch.cat([r[1] for r in res])
            if ref is None:
                ref = ids
            elif rnd == 0:
                print(f"group {v}: ids identical: {bool(torch.equal(ids, ref))}", flush=True)
            print(f"round {rnd} group {v}: {times[v][-1]:.4f} ms/batch", flush=True)
    print(json.dumps({v: {"ms_min": min(t), "ms_mean": sum(t) / len(t), "qps_best": 128 / min(t) * 1e3}
                      for v, t in times.items()}))


if __name__ == "__main__":
    main()
