"""Attention forward A/B, one library per process (DRT_LIB=<variant>): drt_attention_bf16 at the encode
leg's half batch (256 x 128 x 12 heads; all-ones and ragged masks), the query tower's (128 x 32) and a
ragged 64 x 100 -- HIP-event us per launch and an output digest -- then the encode leg (passages/s)."""
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(reps=50):
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    dev = torch.device("cuda", 0)
    st = _native.stream_ptr(dev)
    heads, dh = 12, 64
    H = heads * dh
    res = {"lib": os.path.basename(os.environ.get("DRT_LIB", "product"))}
    g = torch.Generator(device=dev).manual_seed(1)
    shapes = ((256, 128, False), (256, 128, True), (128, 32, False), (64, 100, True))
    if os.environ.get("ATTN_SHAPES") == "rerank":
        shapes = ((500, 160, False), (625, 128, False), (500, 160, True))
    for (B, L, ragged) in shapes:
        qkv = (torch.randn((B * L, 3 * H), generator=g, device=dev) * 2).to(torch.bfloat16)
        mask = torch.ones((B, L), dtype=torch.int64, device=dev)
        if ragged:
            lens = torch.randint(L // 4, L + 1, (B,), generator=g, device=dev)
            mask = (torch.arange(L, device=dev)[None, :] < lens[:, None]).to(torch.int64)
        ctx = torch.empty((B * L, H), dtype=torch.bfloat16, device=dev)
        run = lambda: _native.check(lib.drt_attention_bf16(qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), B, L,
                                                           heads, dh, 1.0 / math.sqrt(dh), st), "attn")
        run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000 / reps)
        nbytes = B * L * 4 * H * 2
        t = sorted(ts)[2]
        res[f"B{B}_L{L}{'_ragged' if ragged else ''}"] = {
            "us": round(t, 2), "hbm_frac": round(nbytes / (t * 1e-6) / 8e12, 3),
            "digest": int(ctx.view(torch.int16).reshape(-1).double().mul(
                torch.arange(ctx.numel(), device=dev, dtype=torch.float64).remainder(997)).sum().item())}
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, dev)
    del m
    B, L = 512, 128
    ids = torch.randint(1000, 30522, (B, L), device=dev, generator=torch.Generator(device=dev).manual_seed(9))
    mask = torch.ones((B, L), dtype=torch.int64, device=dev)
    enc(ids, mask)
    torch.cuda.synchronize()
    pps = []
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(8):
            enc.pool(enc(ids, mask), mask, "first")
        torch.cuda.synchronize()
        pps.append(round(8 * B / (time.perf_counter() - t0), 1))
    res["encode_pps"] = pps
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
