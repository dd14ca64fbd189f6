"""One encoder GEMM shape, one kernel variant, a few launches (for rocprofv3 --pmc passes).
usage: gemm_one.py VARIANT [N K FLAGS [M]]"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from denseretrievaltoolkits_amd import _native  # noqa: E402

v = int(sys.argv[1])
N, K, flags = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (768, 3072, 2)
M = int(sys.argv[5]) if len(sys.argv) > 5 else 65536
lib = _native.load()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
w = (0.05 * torch.randn(N, K, generator=g, device=dev)).to(torch.bfloat16)
b = torch.randn(N, generator=g, device=dev)
r = torch.randn(M, N, generator=g, device=dev).to(torch.bfloat16) if flags & 2 else None
out = torch.empty(M, N, dtype=torch.float32 if flags & 2 else torch.bfloat16, device=dev)
lib.drt_gemm_force_small(v)
s = _native.stream_ptr(dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(2):
    e0.record()
    for _ in range(5):
        _native.check(lib.drt_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(),
                                          r.data_ptr() if r is not None else None, out.data_ptr(), M, N, K, flags, s),
                      "linear")
    e1.record()
    torch.cuda.synchronize()
print(f"variant {v} M={M} N={N} K={K}: {2 * M * N * K / (e0.elapsed_time(e1) / 5) / 1e9:.1f} TFLOP/s")
