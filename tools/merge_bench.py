#!/usr/bin/env python3
"""Microbenchmark of the small post-scan kernels (merge_packed, dist_tau, topk_merge)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseretrievaltoolkits_amd import kernels  # noqa: E402


def timeit(fn, it=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


dev = torch.device("cuda", 0)
for nparts, nq, k in [(8, 128, 1000), (2, 128, 1000), (8, 128, 100), (8, 16, 1000), (4, 128, 1000), (1, 128, 1000)]:
    keys = torch.randint(0, 2**62, (nparts, nq, k + 1), device=dev, dtype=torch.int64)
    keys[:, :, :k] = keys[:, :, :k].sort(dim=2).values
    keys[:, :, k] = 0
    us = timeit(lambda: kernels.merge_packed(keys, k, 10_000_000))
    s = torch.randn(nparts, nq, k, device=dev).sort(dim=2, descending=True).values
    i = torch.randint(0, 10**7, (nparts, nq, k), device=dev)
    us2 = timeit(lambda: kernels.topk_merge(s, i, k))
    print(f"nparts={nparts} nq={nq} k={k}: merge_packed {us:.1f} us, topk_merge {us2:.1f} us", flush=True)
r = kernels.sample_rank(1000)
lists = torch.randint(0, 2**31, (8, 128, r), device=dev, dtype=torch.int32)
print(f"dist_tau 8x128x{r}: {timeit(lambda: kernels.dist_tau(lists, 1000)):.1f} us")
print(f"empty launch (torch fill 1 elem): {timeit(lambda: lists[0, 0, 0].fill_(1)):.1f} us")
