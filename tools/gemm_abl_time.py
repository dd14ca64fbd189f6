#!/usr/bin/env python3
"""Time drt_linear_bf16 on the encoder projection shapes (one half-batch of 32768 tokens, production
epilogues) -- run once per DRT_LIB variant library for ablations (tools/build_variant.sh).
usage: DRT_LIB=... python tools/gemm_abl_time.py [M] [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseretrievaltoolkits_amd import _native  # noqa: E402

SHAPES = [("qkv", 2304, 768, 0, False), ("oproj", 768, 768, 0, True), ("ffn1", 3072, 768, 1, False),
          ("ffn2", 768, 3072, 0, True)]


def main(M=32768, reps=20):
    lib = _native.load()
    dev = torch.device("cuda", 0)
    s = _native.stream_ptr(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    out = {"lib": os.path.basename(os.environ.get("DRT_LIB", "product")), "M": M}
    for name, N, K, flags, resid in SHAPES:
        x = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (0.05 * torch.randn(N, K, generator=g, device=dev)).to(torch.bfloat16)
        b = torch.randn(N, generator=g, device=dev)
        r = torch.randn(M, N, generator=g, device=dev).to(torch.bfloat16) if resid else None
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)

        def call():
            _native.check(lib.drt_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(),
                                              r.data_ptr() if r is not None else None, y.data_ptr(), M, N, K, flags, s),
                          name)
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        # bit checksum of the output, to compare variants that must agree exactly
        crc = int((y.view(torch.int16).to(torch.int64) * torch.arange(1, y.numel() + 1, device=dev).view(M, N)
                   .remainder(65521)).sum())
        out[name] = {"us": round(us, 1), "tflops": round(2 * M * N * K / us / 1e6, 1), "crc": crc}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])
