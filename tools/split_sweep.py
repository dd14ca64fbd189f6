#!/usr/bin/env python3
"""Query-tower forward time (32 tokens) per split-K planning config (drt_gemm_split_config),
batches 128 and 512, interleaved rounds in one process; pooled reps compared with the default."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseretrievaltoolkits_amd import _native  # noqa: E402
from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder  # noqa: E402

CONFIGS = {   # (large_min_k, large_k_per_split, small_cap_bytes)
    "default": (8192, 512, 16 << 20),
    "l2048k512": (2048, 512, 16 << 20),
    "l2048k768": (2048, 768, 16 << 20),
    "l2048k512_s64": (2048, 512, 64 << 20),
    "s64": (8192, 512, 64 << 20),
}


def main():
    from transformers import BertConfig, BertModel
    lib = _native.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    g = torch.Generator(device=dev).manual_seed(4)
    res = {c: {} for c in CONFIGS}
    ref = {}
    for rnd in range(3):
        for name, cfg in CONFIGS.items():
            lib.drt_gemm_split_config(*cfg)
            enc = HipBertEncoder.from_hf(m, dev)
            for B in (128, 512):
                ids = torch.randint(1000, 30522, (B, 32), generator=torch.Generator(device=dev).manual_seed(B),
                                    device=dev, dtype=torch.int64)
                ids[:, 0], ids[:, -1] = 101, 102
                mask = torch.ones_like(ids)
                for _ in range(3):
                    out = enc.pool(enc(ids, mask), mask, "first")[0]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(20):
                    out = enc.pool(enc(ids, mask), mask, "first")[0]
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / 20 * 1e3
                res[name].setdefault(B, []).append(ms)
                if name == "default" and rnd == 0:
                    ref[B] = out.float().clone()
                elif rnd == 0:
                    cos = torch.nn.functional.cosine_similarity(out.float(), ref[B], dim=1).min().item()
                    print(f"{name} B={B}: min cos vs default {cos:.6f}", flush=True)
            del enc
            print(f"round {rnd} {name}: " + ", ".join(f"B{B} {v[-1]:.3f} ms" for B, v in res[name].items()), flush=True)
    lib.drt_gemm_split_config(*CONFIGS["default"])
    print(json.dumps({n: {B: round(min(v), 4) for B, v in r.items()} for n, r in res.items()}))


if __name__ == "__main__":
    main()
