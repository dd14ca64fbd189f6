#!/usr/bin/env python3
"""Microbenchmark of merge_packed's kernels (count / rank / tree) on realistic packed lists:
global-threshold regime (each of W parts holds ~1.3 k / W valid keys, count in entry k) and
the one-part case (k valid keys), for one batch (128 queries) and one group (2048)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseretrievaltoolkits_amd import _native, kernels  # noqa: E402


def timeit(fn, it=30):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


def packed(nparts, nq, k, fill, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(nparts * 7 + nq)
    keys = torch.randint(0, 2**62, (nparts, nq, k + 1), device=dev, dtype=torch.int64, generator=g)
    cnt = min(k, int(fill))
    keys[:, :, :k] = keys[:, :, :k].sort(dim=2).values
    keys[:, :, cnt:k] = -1                      # ~0 = empty
    keys[:, :, k] = cnt << 32
    return keys


lib = _native.load()
dev = torch.device("cuda", 0)
k = 1000
for nparts, fill in [(8, 1.3 * k / 8), (4, 1.3 * k / 4), (2, 1.3 * k / 2), (1, k)]:
    for nq in (128, 2048):
        pk = packed(nparts, nq, k, fill, dev)
        row = []
        ref = None
        for v in (3, 2, 1):
            _native.check(lib.drt_topk_merge_packed_variant(v), "variant")
            us = timeit(lambda: kernels.merge_packed(pk, k, 10_000_000))
            out = kernels.merge_packed(pk, k, 10_000_000)
            if ref is None:
                ref = out
            else:
                assert torch.equal(out[1], ref[1]) and torch.equal(out[2], ref[2]), (nparts, nq, v)
            row.append(f"v{v} {us:7.1f} us")
        print(f"nparts={nparts} nq={nq:5d} valid/part={int(fill):4d}: " + "  ".join(row), flush=True)
_native.check(lib.drt_topk_merge_packed_variant(0), "variant")
