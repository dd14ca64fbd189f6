#!/usr/bin/env python3
"""One-GPU grouped search, chunked: a group of 16 query batches (2048 queries) against the 10M x 768
shard with the filter pass as ONE launch over the whole shard (the product's grouped path) vs one launch
per row chunk of `--chunk` rows (each chunk's packed lists a separate part, merged by merge_packed like
the shards of a multi-GPU index): short launches keep the group's 16 query blocks in step, so a tile
reaches each XCD's L2 once for all of them.  Times the filter passes + the merge only
(sample / threshold once, untimed); checks both give the same ids.
usage: python tools/group_chunk_probe.py [--chunk 1250000] [--reps 3]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--chunk", type=int, default=1_250_000)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from bench import gen_shard
    from denseretrievaltoolkits_amd import kernels
    dev = torch.device("cuda", 0)
    p, _, _ = gen_shard(a.n, 1, 0, 768, dev)
    g = torch.Generator(device=dev).manual_seed(5678)
    q = torch.randn((2048, 768), generator=g, device=dev).to(torch.bfloat16)
    k = a.k
    tau = kernels.dist_tau(kernels.dist_sample(q, p, a.n, k)[None].contiguous(), k)
    chunks = [(c, min(a.n, c + a.chunk)) for c in range(0, a.n, a.chunk)]

    def whole():
        packed = torch.empty((1, 2048, k + 1), dtype=torch.int64, device=dev)
        kernels.dist_filter_into(q, p, a.n, k, 0, tau, packed[0])
        return kernels.merge_packed(packed, k, a.n)

    def chunked():
        packed = torch.empty((len(chunks), 2048, k + 1), dtype=torch.int64, device=dev)
        for j, (c0, c1) in enumerate(chunks):
            kernels.dist_filter_into(q, p[c0:c1], a.n, k, c0, tau, packed[j])
        return kernels.merge_packed(packed, k, a.n)

    out = {"n": a.n, "chunk": a.chunk, "chunks": len(chunks), "queries": 2048}
    ref = None
    for name, fn in (("whole", whole), ("chunked", chunked), ("whole", whole), ("chunked", chunked)):
        r = fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            r = fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        out.setdefault(name + "_ms_per_group", []).append(round(ms, 2))
        if ref is None:
            ref = r
        else:
            out["ids_equal_" + name] = bool(torch.equal(ref[1], r[1]))
            out["status_ok_" + name] = int((r[2] == 0).sum())
    out["ms_per_batch"] = {n: round(min(out[n + "_ms_per_group"]) / 16, 3) for n in ("whole", "chunked")}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
