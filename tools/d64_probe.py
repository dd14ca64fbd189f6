import sys, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from helpers import int_bf16
from oracle import search_oracle as orc
from denseretrievaltoolkits_amd import kernels
dev = torch.device('cuda', 0)
for name, dd, n, k, lo in (("d8pad", 8, 20011, 50, -3), ("d64full", 64, 20011, 50, -3), ("d64_n1000", 8, 1000, 50, -3),
                           ("d8pad_big", 8, 200011, 50, -3), ("d128_8", 8, 20011, 50, -3)):
    rng = np.random.default_rng(8)
    D = 128 if name == "d128_8" else 64
    p = np.zeros((n, D), np.float32); q = np.zeros((37, D), np.float32)
    p[:, :dd] = int_bf16(rng, (n, dd), lo, 3); q[:, :dd] = int_bf16(rng, (37, dd), lo, 3)
    es, ei = orc.ip_topk(q, p, k)
    qd = torch.from_numpy(q).to(torch.bfloat16).to(dev); pd = torch.from_numpy(p).to(torch.bfloat16).to(dev)
    s, i, st = kernels.ip_topk(qd, pd, k, resolve=False)
    s, i, st = s.cpu().numpy(), i.cpu().numpy(), st.cpu().numpy()
    bad = [(r, ) for r in range(37) if not np.array_equal(i[r], ei[r])]
    print(name, "status", np.unique(st, return_counts=True), "rows wrong", len(bad), flush=True)
    if bad:
        r = bad[0][0]
        print("  row", r, "gpu", i[r][:8], s[r][:8], "ref", ei[r][:8], es[r][:8], flush=True)
    s2, i2, st2 = kernels.ip_topk(qd, pd, k, resolve=True)
    print("  resolved wrong rows", sum(not np.array_equal(i2.cpu().numpy()[r], ei[r]) for r in range(37)), flush=True)
