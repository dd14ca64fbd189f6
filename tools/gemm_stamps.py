"""Segment stamps (s_memtime) of the ping-pong GEMM, variant 6 (diagnostic build of
variant 3): per slab and wave, the cycles of each part of the four barrier-delimited
segments (slabs 8-11 of the first tile of blocks 0-15)."""
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
dbg = torch.zeros(16 * 8 * 4 * 10, dtype=torch.int64, device=dev)
lib.drt_gemm_debug_buffer(dbg.data_ptr())
lib.drt_gemm_force_small(6)
s = _native.stream_ptr(dev)
for _ in range(4):
    _native.check(lib.drt_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(), r.data_ptr() if r is not None else None,
                                      out.data_ptr(), M, N, K, flags, s), "linear")
torch.cuda.synchronize()
t = dbg.cpu().numpy().reshape(16, 8, 4, 10).astype(np.int64)
names = ["A.wait_lgkm", "A.mfma_issue", "A.bar", "Bm.issue", "Bm.bar", "B.wait_lgkm", "B.mfma_issue", "B.bar",
         "Am.issue", "Am.bar"]
rows = []
for sl in range(3):
    cur, nxt = t[:, :, sl], t[:, :, sl + 1]
    seq = [cur[..., 1] - cur[..., 0], cur[..., 2] - cur[..., 1], cur[..., 3] - cur[..., 2],
           cur[..., 4] - cur[..., 3], cur[..., 5] - cur[..., 4], cur[..., 6] - cur[..., 5],
           cur[..., 7] - cur[..., 6], nxt[..., 8] - cur[..., 7], nxt[..., 9] - nxt[..., 8], nxt[..., 0] - nxt[..., 9]]
    rows.append(np.stack(seq, -1))
d = np.concatenate(rows, 0)  # [48, 8, 10]
for g, wv in (("waves 0-3", slice(0, 4)), ("waves 4-7", slice(4, 8))):
    med = np.median(d[:, wv], axis=(0, 1))
    print(g, " ".join(f"{n}={int(v)}" for n, v in zip(names, med)), "slab=", int(med.sum()))
