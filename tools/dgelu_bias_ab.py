"""FFN1 dgrad + bias gradient at the recipe passage shape (T = 1024 x 156, N = 3072, K = 768): the
fused entry (drt_linear_dgelu_bias_bf16: column sums from the GEMM epilogue) vs the dgrad
(drt_linear_bf16_ex with gelu_pre) followed by drt_colsum_bf16 over dX, interleaved, HIP events."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseretrievaltoolkits_amd import _native  # noqa: E402


def main(reps=20):
    lib = _native.load()
    dev = torch.device("cuda", 0)
    s = _native.stream_ptr(dev)
    res = {}
    for T in (159744, 131072, 16384):
        N, K = 3072, 768
        g = torch.Generator(device=dev).manual_seed(1)
        dy = torch.randn(T, K, generator=g, device=dev).to(torch.bfloat16)
        wt = (0.05 * torch.randn(N, K, generator=g, device=dev)).to(torch.bfloat16)
        pre = torch.randn(T, N, generator=g, device=dev).to(torch.bfloat16)
        dx = torch.empty(T, N, dtype=torch.bfloat16, device=dev)
        db = torch.empty(N, device=dev)
        nbf = int(lib.drt_linear_dgelu_bias_workspace(T, N, K))
        wsf = torch.empty(max(1, nbf // 4 + 1), device=dev)
        nbl = int(lib.drt_linear_workspace(T, N, K))
        wsl = torch.empty(max(1, nbl // 4 + 1), device=dev)
        nbc = int(lib.drt_colsum_workspace(T, N))
        wsc = torch.empty(max(1, nbc // 4 + 1), device=dev)

        def fused():
            lib.drt_linear_dgelu_bias_bf16(dy.data_ptr(), wt.data_ptr(), pre.data_ptr(), dx.data_ptr(), T, N, K,
                                           db.data_ptr(), wsf.data_ptr(), nbf, s)

        def unfused():
            lib.drt_linear_bf16_ex(dy.data_ptr(), wt.data_ptr(), None, None, pre.data_ptr(), dx.data_ptr(), None, T,
                                   N, K, 0, 0.0, 0, 0, wsl.data_ptr(), nbl, s)
            lib.drt_colsum_bf16(dx.data_ptr(), T, N, db.data_ptr(), wsc.data_ptr(), nbc, s)

        def gemm_only():
            lib.drt_linear_bf16_ex(dy.data_ptr(), wt.data_ptr(), None, None, pre.data_ptr(), dx.data_ptr(), None, T,
                                   N, K, 0, 0.0, 0, 0, wsl.data_ptr(), nbl, s)
        out = {}
        for _ in range(2):
            for name, fn in (("fused", fused), ("unfused", unfused), ("gemm_only", gemm_only)):
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                out.setdefault(name, []).append(round(e0.elapsed_time(e1) / reps * 1e3, 1))
        res[f"T{T}"] = out
    print(json.dumps(res))


if __name__ == "__main__":
    main()
