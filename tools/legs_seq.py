#!/usr/bin/env python3
"""The bench's model legs in bench order in one process, with the allocator state after each, and the
recipe step timed at the end (and optionally first): finds which earlier leg slows the recipe leg
(r04s: 169 ms in the full bench vs 119 alone).  usage: python tools/legs_seq.py [--first]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", default="encode,rerank,query,scores,train")
    args = ap.parse_args()
    import bench_legs as bl
    dev = torch.device("cuda", 0)

    def mem(tag):
        st = torch.cuda.memory_stats(dev)
        print(json.dumps({"after": tag, "reserved_gb": round(torch.cuda.memory_reserved(dev) / 2**30, 1),
                          "allocated_gb": round(torch.cuda.memory_allocated(dev) / 2**30, 2),
                          "alloc_retries": st.get("num_alloc_retries", 0),
                          "segments": st.get("segment.all.current", 0)}), flush=True)

    def recipe(tag):
        t0 = time.perf_counter()
        r = bl.run_train_step(dev, bq=128, n=8, p_len=156, steps=3, warmup=1)
        print(json.dumps({"recipe_" + tag: r["hip_ms"], "torch_bf16": r["torch_bf16_autocast_ms"],
                          "leg_s": round(time.perf_counter() - t0, 1)}), flush=True)

    def search_leg():   # bench.py's search leg + its CPU baseline, corpus dropped afterwards
        import types
        import bench
        from denseretrievaltoolkits_amd.search import FlatIPIndex
        shard, _, _ = bench.gen_shard(10_000_000, 1, 0, 768, dev)
        g = torch.Generator(device=dev)
        g.manual_seed(1234)
        qs = [torch.randn((128, 768), generator=g, device=dev).to(torch.bfloat16) for _ in range(20)]
        idx = FlatIPIndex.from_rows(shard)
        res = idx.search_batches(qs, 1000)
        torch.cuda.synchronize()
        a = types.SimpleNamespace(n_corpus=10_000_000, k=1000, qb=128, dim=768)
        bench.cpu_baseline(a, shard, qs[0], res[0])
        del shard, qs, idx, res

    def cpu_leg():
        import bench
        bench.encode_cpu_baseline()

    legs = {"search": search_leg, "cpu": cpu_leg,
            "encode": lambda: bl.run(dev), "rerank": lambda: bl.run_rerank(dev),
            "query": lambda: bl.run_query_encode(dev), "scores": lambda: bl.run_train_scores(dev),
            "train": lambda: bl.run_train_step(dev)}
    for name in args.legs.split(","):
        legs[name]()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        mem(name)
        if name in ("search", "cpu", "encode", "query", "train"):
            recipe("after_" + name)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
