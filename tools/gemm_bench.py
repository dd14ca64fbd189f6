"""GEMM throughput of the encoder projection shapes: large-tile vs 128^2 kernel (HIP events)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from denseretrievaltoolkits_amd import _native  # noqa: E402


def run():
    lib = _native.load()
    dev = torch.device("cuda", 0)
    M = 65536
    shapes = [("qkv", 2304, 768, 0), ("oproj", 768, 768, 2), ("ffn1", 3072, 768, 1), ("ffn2", 768, 3072, 2)]
    res = {}
    for name, N, K, flags in shapes:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev).to(torch.bfloat16) if flags & 2 else None
        out = torch.empty(M, N, dtype=torch.float32 if flags & 2 else torch.bfloat16, device=dev)
        for force in (0, 1, 2):
            lib.drt_gemm_force_small(force)
            s = _native.stream_ptr(dev)
            call = lambda: lib.drt_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(),
                                               r.data_ptr() if r is not None else None, out.data_ptr(), M, N, K,
                                               flags, s)
            for _ in range(3):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            n = 20
            for _ in range(n):
                call()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            res[f"{name}_{['large', 'small', 'half'][force]}"] = round(2 * M * N * K / ms / 1e9, 1)
        # hipBLASLt reference point (torch.matmul, bf16 out, no epilogue)
        for _ in range(3):
            y = x @ w.T
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            y = x @ w.T
        e1.record()
        torch.cuda.synchronize()
        res[f"{name}_torch"] = round(2 * M * N * K / (e0.elapsed_time(e1) / 20) / 1e9, 1)
    lib.drt_gemm_force_small(0)
    print(json.dumps({"gemm_tflops": res}))


if __name__ == "__main__":
    run()
