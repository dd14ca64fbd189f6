"""GEMM throughput of the encoder projection shapes per kernel variant (HIP events),
plus a correctness check of every variant against torch fp32 and torch's hipBLASLt
bf16 GEMM as a reference point.  Variants: 0 auto (= 8), 1 128^2, 2 large half-K ring,
7/8 ping-pong 256^2 with a 4/5-slot ring, 9 full-K 32x32x16 256^2."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from denseretrievaltoolkits_amd import _native  # noqa: E402

VARIANTS = {0: "auto", 1: "small", 2: "half", 7: "pp1", 8: "pp1r5", 9: "large32"}


def run(M=65536, reps=20, variants=(0, 1, 2, 3)):
    lib = _native.load()
    dev = torch.device("cuda", 0)
    shapes = [("qkv", 2304, 768, 0), ("oproj", 768, 768, 2), ("ffn1", 3072, 768, 1), ("ffn2", 768, 3072, 2)]
    res, err = {}, {}
    g = torch.Generator(device=dev).manual_seed(0)
    for name, N, K, flags in shapes:
        x = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (0.05 * torch.randn(N, K, generator=g, device=dev)).to(torch.bfloat16)
        b = torch.randn(N, generator=g, device=dev)
        r = torch.randn(M, N, generator=g, device=dev).to(torch.bfloat16) if flags & 2 else None
        ref = x.float() @ w.float().T + b
        if flags & 1:
            ref = torch.nn.functional.gelu(ref)
        if r is not None:
            ref += r.float()
        out = torch.empty(M, N, dtype=torch.float32 if flags & 2 else torch.bfloat16, device=dev)
        for v in variants:
            lib.drt_gemm_force_small(v)
            s = _native.stream_ptr(dev)
            call = lambda: lib.drt_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(),
                                               r.data_ptr() if r is not None else None, out.data_ptr(), M, N, K,
                                               flags, s)
            out.zero_()
            _native.check(call(), "linear")
            torch.cuda.synchronize()
            err[f"{name}_{VARIANTS[v]}"] = float((out.float() - ref).abs().max())
            for _ in range(3):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                call()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            res[f"{name}_{VARIANTS[v]}"] = round(2 * M * N * K / ms / 1e9, 1)
        for _ in range(3):
            y = x @ w.T
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            y = x @ w.T
        e1.record()
        torch.cuda.synchronize()
        res[f"{name}_torch"] = round(2 * M * N * K / (e0.elapsed_time(e1) / reps) / 1e9, 1)
        del y
    lib.drt_gemm_force_small(0)
    print(json.dumps({"gemm_tflops": res, "max_abs_err": err}))


if __name__ == "__main__":
    vs = tuple(int(v) for v in sys.argv[1].split(",")) if len(sys.argv) > 1 else (0, 1, 9)
    orders = tuple(int(v) for v in sys.argv[2].split(",")) if len(sys.argv) > 2 else (-1,)
    for o in orders:
        _native.load().drt_gemm_tile_order(o)
        print("tile order", o)
        run(variants=vs)
