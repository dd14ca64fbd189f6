#!/usr/bin/env python3
"""Weight-gradient GEMM dW = dY^T X at the C3 passage-tower shapes (T = 1024 x 128 tokens):
TN kernel straight from the token-major operands vs the transposed path (2 transposes + NT
GEMM), HIP events around each, TF/s of the GEMM flops."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(T=131072, reps=10):
    import torch
    from denseretrievaltoolkits_amd.model import encoder_bwd as eb
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for name, N, K in [("qkv", 2304, 768), ("oproj", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)]:
        x = torch.randn(T, K, generator=g, device=dev).to(torch.bfloat16)
        dy = torch.randn(T, N, generator=g, device=dev).to(torch.bfloat16)
        for mode in (True, False):
            eb.WGRAD_TN = mode
            for _ in range(2):
                eb.wgrad(dy, x)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                eb.wgrad(dy, x)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            res[f"{name}_{'tn' if mode else 'transposed'}"] = {"ms": round(ms, 4),
                                                               "tflops": round(2 * T * N * K / ms / 1e9, 1)}
        eb.WGRAD_TN = True
    print(json.dumps(res))


if __name__ == "__main__":
    main()
