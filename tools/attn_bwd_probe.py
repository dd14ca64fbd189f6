"""Attention forward / backward at the C3 passage shape (1024 x 128, 12 heads) and the recipe
shape (1024 x 156): time with and without attention-probability dropout (HIP events), and the
memory floor of each (bytes read + written / 6.3 TB/s)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseretrievaltoolkits_amd import _native  # noqa: E402


def main(reps=10, shapes=((1024, 128), (1024, 156), (512, 32))):
    lib = _native.load()
    dev = torch.device("cuda", 0)
    s = _native.stream_ptr(dev)
    res = {}
    torch.manual_seed(0)
    for B, L in shapes:
        H, heads = 768, 12
        T = B * L
        qkv = (0.5 * torch.randn(T, 3 * H, device=dev)).to(torch.bfloat16)
        ctx = torch.empty(T, H, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(B * heads * L, dtype=torch.float32, device=dev)
        dctx = (0.1 * torch.randn(T, H, device=dev)).to(torch.bfloat16)
        dqkv = torch.empty_like(qkv)
        mask = torch.ones(B, L, dtype=torch.int64, device=dev)
        bits = torch.empty((B, heads, L, (L + 31) // 32), dtype=torch.int32, device=dev)
        # L > 160 (streamed backward): dropout needs the forward's bits, no hash variant
        for p, use_bits in ((0.0, False), (0.1, True)) + (((0.1, False),) if L <= 160 else ()):
            bp = bits.data_ptr() if use_bits else None

            def fwd():
                return lib.drt_attention_train_fwd_bits_bf16(qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(),
                                                             lse.data_ptr(), bp, B, L, heads, 64, 0.125, p, 123, 4, s)

            def bwd():
                return lib.drt_attention_train_bwd_bits_bf16(qkv.data_ptr(), ctx.data_ptr(), dctx.data_ptr(),
                                                             lse.data_ptr(), mask.data_ptr(), bp, dqkv.data_ptr(), B,
                                                             L, heads, 64, 0.125, p, 123, 4, s)
            tag = "" if p == 0 else ("_bits" if use_bits else "_hash")
            for name, fn in (("fwd", fwd), ("bwd", bwd)):
                _native.check(fn(), name)
                _native.check(fn(), name)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[f"B{B}_L{L}_{name}_p{p}{tag}"] = round(e0.elapsed_time(e1) / reps * 1e3, 1)
                if name == "bwd":   # position-weighted checksum of dQKV: variants compare bitwise
                    v = dqkv.view(torch.int16).view(-1).long()
                    w = torch.arange(v.numel(), device=dev) % 1009 + 1
                    res[f"B{B}_L{L}_bwd_p{p}{tag}_sum"] = int((v * w).sum())
                    del v, w
        fwd_bytes = T * 3 * H * 2 + T * H * 2
        bwd_bytes = T * 3 * H * 2 + 2 * T * H * 2 + T * 3 * H * 2
        res[f"B{B}_L{L}_floor_us"] = {"fwd": round(fwd_bytes / 6.3e12 * 1e6, 1), "bwd": round(bwd_bytes / 6.3e12 * 1e6, 1)}
        # matrix flops: forward S, PV; backward S, dP, dV, dK, dQ (the streamed L > 160 kernels recompute
        # S and dP in the dQ pass: 7 products)
        per = 2 * L * L * 64 * heads * B
        res[f"B{B}_L{L}_gflop"] = {"fwd": round(2 * per / 1e9, 1), "bwd": round((5 if L <= 160 else 7) * per / 1e9, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    # usage: attn_bwd_probe.py [reps] [BxL,BxL,...]
    shp = tuple(tuple(int(v) for v in x.split("x")) for x in sys.argv[2].split(",")) if len(sys.argv) > 2 else None
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10, *((shp,) if shp else ()))
