#!/usr/bin/env python3
"""Time kernels.ip_topk's large-k path (k > 2048) against the k = 1000 / 2048 list kernels on one
device-generated Gaussian corpus (default 10M x 768 bf16, 128 queries), canonical order both ways.
usage: python tools/large_k_probe.py [n] [nq]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseretrievaltoolkits_amd import kernels  # noqa: E402


def main(n=10_000_000, nq=128):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    p = torch.empty((n, 768), dtype=torch.bfloat16, device=dev)
    for a in range(0, n, 1 << 20):
        b = min(n, a + (1 << 20))
        p[a:b] = torch.randn((b - a, 768), generator=g, device=dev).to(torch.bfloat16)
    q = torch.randn((nq, 768), generator=g, device=dev).to(torch.bfloat16)
    stats = kernels.row_stats(p)
    out = {"n": n, "nq": nq}
    for k in (1000, 2048, 4096, 8192, 32768):
        kernels.ip_topk(q, p, k, stats=stats)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            s, i, st = kernels.ip_topk(q, p, k, stats=stats)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        out[f"k{k}"] = {"ms": round(ms, 2), "queries_per_s": round(nq / ms * 1e3, 1),
                        "status_nonzero": int((st != 0).sum())}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])
