"""LayerNorm A/B (run once per library, DRT_LIB=<variant>): drt_layernorm_bf16 at the encoder's
half-batch shape (32768 x 768 bf16) -- HIP-event time per launch and an output digest -- then the
encode leg (512 x 128 passages/s)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(reps=100):
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    dev = torch.device("cuda", 0)
    st = _native.stream_ptr(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    res = {"lib": os.path.basename(os.environ.get("DRT_LIB", "product"))}
    for M in (32768, 4096, 100):
        H = 768
        x = (torch.randn((M, H), generator=g, device=dev) * 3 + 0.5).to(torch.bfloat16)
        gam = torch.rand(H, generator=g, device=dev) + 0.5
        bet = torch.randn(H, generator=g, device=dev)
        out = torch.empty_like(x)
        run = lambda: _native.check(lib.drt_layernorm_bf16(x.data_ptr(), M, H, gam.data_ptr(), bet.data_ptr(),
                                                           1e-12, out.data_ptr(), st), "ln")
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
        ref = torch.nn.functional.layer_norm(x.float(), (H,), gam, bet, 1e-12)
        res[f"M{M}"] = {"us": round(sorted(ts)[2], 2), "tb_s": round(4 * M * H / (sorted(ts)[2] * 1e-6) / 1e12, 2),
                        "digest": int(out.view(torch.int16).reshape(-1).double().mul(torch.arange(out.numel(), device=dev,
                                      dtype=torch.float64).remainder(997)).sum().item()),
                        "max_abs_vs_torch_fp32": round(float((out.float() - ref).abs().max()), 4)}
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, dev)
    del m
    B, L = 512, 128
    ids = torch.randint(1000, 30522, (B, L), device=dev, generator=torch.Generator(device=dev).manual_seed(9))
    mask = torch.ones((B, L), dtype=torch.int64, device=dev)
    h = enc(ids, mask)
    torch.cuda.synchronize()
    res["encode_digest"] = int(h.view(torch.int16)[:, 0, :].double().sum().item())
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
