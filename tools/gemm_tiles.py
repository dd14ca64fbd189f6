"""Per-tile timeline of the pp1 GEMM (diagnostic variant 31: wave-0 stamps at kernel
start, loop start, loop end, epilogue end + XCC/HW ids): prologue / loop / epilogue
cycles and the gaps between consecutive tiles on one CU."""
import os
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseretrievaltoolkits_amd import _native  # noqa: E402

N, K, flags = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (2304, 768, 0)
M = 65536
lib = _native.load()
dev = torch.device("cuda", 0)
x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
w = (0.05 * torch.randn(N, K, device=dev)).to(torch.bfloat16)
b = torch.randn(N, device=dev)
r = torch.randn(M, N, device=dev).to(torch.bfloat16) if flags & 2 else None
out = torch.empty(M, N, dtype=torch.float32 if flags & 2 else torch.bfloat16, device=dev)
tiles = (M // 256) * (N // 256)
dbg = torch.zeros(tiles * 6, dtype=torch.int64, device=dev)
lib.drt_gemm_debug_buffer(dbg.data_ptr())
lib.drt_gemm_force_small(31)
s = _native.stream_ptr(dev)
for _ in range(5):
    _native.check(lib.drt_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(), r.data_ptr() if r is not None else None,
                                      out.data_ptr(), M, N, K, flags, s), "linear")
torch.cuda.synchronize()
lib.drt_gemm_force_small(0)
t = dbg.cpu().numpy().reshape(tiles, 6).astype(np.int64)
t0 = t[:, 0].min()
pro, loop, epi = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
print(f"tiles {tiles}: span {t[:, 3].max() - t0} cycles; median prologue {np.median(pro):.0f} loop {np.median(loop):.0f} "
      f"({np.median(loop) / (K // 32):.0f}/slab) epilogue {np.median(epi):.0f}")
print("prologue pct 10/50/90:", np.percentile(pro, [10, 50, 90]).astype(int), " loop:", np.percentile(loop, [10, 50, 90]).astype(int),
      " epi:", np.percentile(epi, [10, 50, 90]).astype(int))
cu = defaultdict(list)
for i in range(tiles):
    # HW_ID: wave_id[3:0] simd_id[5:4] ... cu_id[11:8] sh_id[12] se_id[15:13] (gfx9 layout)
    key = (int(t[i, 4]), int(t[i, 5]) >> 8 & 0xFF)
    cu[key].append((t[i, 0], t[i, 3]))
gaps = []
for v in cu.values():
    v.sort()
    gaps += [v[j + 1][0] - v[j][1] for j in range(len(v) - 1)]
print(f"CUs seen {len(cu)}, tiles per CU median {np.median([len(v) for v in cu.values()])}; "
      f"gap between tiles on a CU pct 10/50/90: {np.percentile(gaps, [10, 50, 90]).astype(int) if gaps else None}")
# first wave vs later waves of tiles
order = np.argsort(t[:, 0])
first = order[:256]
late = order[-256:]
print("first 256 tiles: loop/slab", np.median(loop[first]) / (K // 32), "prologue", np.median(pro[first]),
      "| last 256: loop/slab", np.median(loop[late]) / (K // 32), "prologue", np.median(pro[late]))
