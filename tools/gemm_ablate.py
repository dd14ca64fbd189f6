"""Loop-only cycle stamps of the pp1 GEMM under ablations (diagnostic variants 16+bits:
1 no LDS-DMA in the loop, 13 = no DMA, no barriers, no fragment reads: the bare MFMA loop,
7 the 5-slot ring with stamps, 10 = LDS-DMA only (no MFMA, no fragment reads)).  Prints
median cycles per slab (first tile of blocks 0-63) and the kernel's TFLOP/s."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseretrievaltoolkits_amd import _native  # noqa: E402

N, K, flags = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (768, 3072, 2)
M = 65536
lib = _native.load()
dev = torch.device("cuda", 0)
x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
w = (0.05 * torch.randn(N, K, device=dev)).to(torch.bfloat16)
b = torch.randn(N, device=dev)
r = torch.randn(M, N, device=dev).to(torch.bfloat16) if flags & 2 else None
out = torch.empty(M, N, dtype=torch.float32 if flags & 2 else torch.bfloat16, device=dev)
dbg = torch.zeros(64 * 8 * 2, dtype=torch.int64, device=dev)
lib.drt_gemm_debug_buffer(dbg.data_ptr())
s = _native.stream_ptr(dev)
names = {0: "base", 1: "nodma", 13: "nods+nobar+nodma", 7: "ring5", 10: "ring5 dma-only"}
for abl, nm in names.items():
    lib.drt_gemm_force_small(16 + abl)
    call = lambda: _native.check(lib.drt_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(),
                                                     r.data_ptr() if r is not None else None, out.data_ptr(),
                                                     M, N, K, flags, s), "linear")
    for _ in range(3):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        call()
    e1.record()
    torch.cuda.synchronize()
    tf = 2 * M * N * K / (e0.elapsed_time(e1) / 10) / 1e9
    t = dbg.cpu().numpy().reshape(64, 8, 2).astype(np.int64)
    cyc = np.median((t[..., 1] - t[..., 0]) / (K // 32))
    print(f"{nm:>20s}: {cyc:7.0f} cycles/slab  {tf:7.1f} TFLOP/s")
lib.drt_gemm_force_small(0)
