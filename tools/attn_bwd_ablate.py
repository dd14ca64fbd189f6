"""Diagnostic: attention backward at the C3 passage shape (1024 x 128, 12 heads, no dropout) per
ablation (drt_attention_force4(16 + ABL): 1 no phase 2, 2 no phase 1, 4 no softmax exp, 8 no P/dS
scratch stores, 12 = 4 + 8), HIP events, interleaved rounds."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseretrievaltoolkits_amd import _native  # noqa: E402


def main(reps=10, rounds=3):
    lib = _native.load()
    dev = torch.device("cuda", 0)
    s = _native.stream_ptr(dev)
    B, L, H, heads = 1024, 128, 768, 12
    T = B * L
    qkv = (0.5 * torch.randn(T, 3 * H, device=dev)).to(torch.bfloat16)
    ctx = torch.empty(T, H, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * heads * L, dtype=torch.float32, device=dev)
    dctx = (0.1 * torch.randn(T, H, device=dev)).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    mask = torch.ones(B, L, dtype=torch.int64, device=dev)
    _native.check(lib.drt_attention_train_fwd_bf16(qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), lse.data_ptr(),
                                                   B, L, heads, 64, 0.125, 0.0, 1, 1, s), "fwd")
    res = {}
    for _ in range(rounds):
        for v in (0, 17, 18, 20, 24, 28):
            _native.check(lib.drt_attention_force4(v), "abl")
            fn = lambda: lib.drt_attention_train_bwd_bf16(qkv.data_ptr(), ctx.data_ptr(), dctx.data_ptr(),
                                                          lse.data_ptr(), mask.data_ptr(), dqkv.data_ptr(), B, L,
                                                          heads, 64, 0.125, 0.0, 1, 1, s)
            _native.check(fn(), "bwd")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(f"abl{max(0, v - 16)}", []).append(round(e0.elapsed_time(e1) / reps * 1e3, 1))
    lib.drt_attention_force4(0)
    print(json.dumps({k: sorted(v)[len(v) // 2] for k, v in res.items()}))


if __name__ == "__main__":
    main()
