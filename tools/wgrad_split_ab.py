#!/usr/bin/env python3
"""Weight-gradient TN GEMM (dW = dY^T X) per split plan, interleaved rounds (HIP events): the
one-round plan (floor(CUs / tiles) splits, default) vs the old ceiling plan (drt_gemm_force_small(14)),
at the C3 passage (T = 131072) and query (T = 16384) tower token counts; outputs compared in fp32
(different split boundaries reorder the fp32 partial sums)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(reps=10, rounds=3):
    import torch
    from denseretrievaltoolkits_amd import _native
    from denseretrievaltoolkits_amd.model import encoder_bwd as eb
    lib = _native.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for T in (131072, 16384):
        for name, N, K in [("qkv", 2304, 768), ("oproj", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)]:
            x = torch.randn(T, K, generator=g, device=dev).to(torch.bfloat16)
            dy = torch.randn(T, N, generator=g, device=dev).to(torch.bfloat16)
            outs, times = {}, {0: [], 14: []}
            for _ in range(rounds):
                for v in (0, 14):
                    lib.drt_gemm_force_small(v)
                    outs[v] = eb.wgrad(dy, x)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(reps):
                        eb.wgrad(dy, x)
                    e1.record()
                    torch.cuda.synchronize()
                    times[v].append(e0.elapsed_time(e1) / reps)
            lib.drt_gemm_force_small(0)
            rel = float((outs[0] - outs[14]).abs().max() / outs[14].abs().max())
            for v in (0, 14):
                ms = sorted(times[v])[rounds // 2]
                res[f"T{T}_{name}_{'one_round' if v == 0 else 'ceil'}"] = {
                    "ms": round(ms, 4), "tflops": round(2 * T * N * K / ms / 1e9, 1)}
            res[f"T{T}_{name}_max_rel_diff"] = rel
    print(json.dumps(res))


if __name__ == "__main__":
    main()
