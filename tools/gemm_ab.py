"""The encoder GEMMs (drt_linear_bf16 with their production epilogues) against torch's hipBLASLt
bf16 GEMM without epilogue on the encoder projection shapes (HIP events, one process, rounds
alternate the two).
usage: python tools/gemm_ab.py [M, default 65536] [rounds]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseretrievaltoolkits_amd import _native  # noqa: E402

SHAPES = [("qkv", 2304, 768, 0, False), ("oproj", 768, 768, 0, True), ("ffn1", 3072, 768, 1, False),
          ("ffn2", 768, 3072, 0, True)]


def main(M=65536, rounds=5, reps=10):
    variants = (0,)
    lib = _native.load()
    dev = torch.device("cuda", 0)
    s = _native.stream_ptr(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for name, N, K, flags, resid in SHAPES:
        x = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (0.05 * torch.randn(N, K, generator=g, device=dev)).to(torch.bfloat16)
        b = torch.randn(N, generator=g, device=dev)
        r = torch.randn(M, N, generator=g, device=dev).to(torch.bfloat16) if resid else None
        outs = {v: torch.empty(M, N, dtype=torch.bfloat16, device=dev) for v in variants}

        def call(v):
            return lib.drt_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(), r.data_ptr() if r is not None else None,
                                       outs[v].data_ptr(), M, N, K, flags, s)

        for v in variants:
            _native.check(call(v), f"{name} v{v}")
        torch.cuda.synchronize()
        times = {v: [] for v in variants}
        tv = ["torch", "torch_bias"] + (["torch_resid_c"] if r is not None else [])
        for t in tv:
            times[t] = []
        for _ in range(rounds):
            for v in list(variants) + tv:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if v == "torch":
                    e0.record()
                    for _ in range(reps):
                        y = x @ w.T
                    e1.record()
                elif v == "torch_bias":   # hipBLASLt with its bias epilogue
                    e0.record()
                    for _ in range(reps):
                        y = torch.nn.functional.linear(x, w, b.to(torch.bfloat16))
                    e1.record()
                elif v == "torch_resid_c":   # hipBLASLt with the residual as C (beta = 1)
                    e0.record()
                    for _ in range(reps):
                        y = torch.addmm(r, x, w.T)
                    e1.record()
                else:
                    e0.record()
                    for _ in range(reps):
                        call(v)
                    e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / reps)
        for v, ts in times.items():
            ts = sorted(ts)
            ms = ts[len(ts) // 2]
            res[f"{name}_{v}"] = {"us": round(ms * 1e3, 1), "tflops": round(2 * M * N * K / ms / 1e9, 1)}
    print(json.dumps({"M": M, "gemm": res}))


if __name__ == "__main__":
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    main(M, rounds)
