#!/usr/bin/env python3
"""Interleaved A/B of search.GROUP_CHUNK_ROWS on the headline workload (10M x 768 bf16, batches of 128,
k 1000, groups of 2048): FlatIPIndex.search_batches end to end (certified, canonical), one process.
usage: python tools/chunk_rows_ab.py [--chunks 1250000,2500000,5000000] [--rounds 3] [--steps 32]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="1250000,2500000,5000000")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--n", type=int, default=10_000_000)
    a = ap.parse_args()
    import torch
    from bench import gen_shard
    from denseretrievaltoolkits_amd import search as srch
    dev = torch.device("cuda", 0)
    shard, _, _ = gen_shard(a.n, 1, 0, 768, dev)
    g = torch.Generator(device=dev).manual_seed(5678)
    qs = torch.randn((a.steps, 128, 768), generator=g, device=dev).to(torch.bfloat16)
    idx = srch.FlatIPIndex.from_rows(shard)
    batches = [qs[j] for j in range(a.steps)]
    ref = None
    for rnd in range(a.rounds):
        for c in [int(x) for x in a.chunks.split(",")]:
            srch.GROUP_CHUNK_ROWS = c
            idx.search_batches(batches[:16], 1000)   # warm (same chunking)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = idx.search_batches(batches, 1000)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            ids = torch.cat([r[1] for r in res])
            if ref is None:
                ref = ids
            same = bool(torch.equal(ids, ref))
            print(json.dumps({"round": rnd, "chunk_rows": c, "ms_per_batch": round(el / a.steps * 1e3, 4),
                              "qps": round(a.steps * 128 / el, 1), "ids_equal_first": same}), flush=True)


if __name__ == "__main__":
    main()
