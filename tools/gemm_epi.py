"""Epilogue cost of the encoder GEMMs (auto kernel, M = 65536 tokens): the same shape with
different epilogues (HIP events).  flags: 1 GELU, 2 fp32 out; 'r' = bf16 residual."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseretrievaltoolkits_amd import _native  # noqa: E402


def main(M=65536, reps=20, variant=0):
    lib = _native.load()
    lib.drt_gemm_force_small(variant)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    cases = [("qkv_bias", 2304, 768, 0, True, False), ("qkv_none", 2304, 768, 0, False, False),
             ("ffn1_gelu", 3072, 768, 1, True, False), ("ffn1_bias", 3072, 768, 0, True, False),
             ("ffn1_none", 3072, 768, 0, False, False),
             ("oproj_b16r", 768, 768, 0, True, True), ("oproj_bias", 768, 768, 0, True, False),
             ("ffn2_b16r", 768, 3072, 0, True, True), ("ffn2_bias", 768, 3072, 0, True, False)]
    res = {}
    s = _native.stream_ptr(dev)
    for name, N, K, flags, bias, resid in cases:
        x = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (0.05 * torch.randn(N, K, generator=g, device=dev)).to(torch.bfloat16)
        b = torch.randn(N, generator=g, device=dev)
        r = torch.randn(M, N, generator=g, device=dev).to(torch.bfloat16) if resid else None
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        call = lambda: lib.drt_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr() if bias else None,
                                           r.data_ptr() if r is not None else None, out.data_ptr(), M, N, K, flags, s)
        for _ in range(3):
            _native.check(call(), name)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        res[name] = {"us": round(ms * 1e3, 1), "tflops": round(2 * M * N * K / ms / 1e9, 1)}
    lib.drt_gemm_force_small(0)
    print(json.dumps({"variant": variant, "epi": res}))


if __name__ == "__main__":
    for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0"]):
        main(variant=int(v))
