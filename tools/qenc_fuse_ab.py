"""Query tower (32 tokens, eager) with and without one of HipBertEncoder's boolean fusion switches
(default fuse_ln: dense + residual + LayerNorm in one call; round 5 also A/B'd a fuse_attn patch, see
DESIGN §1), interleaved rounds, ms per batch.  usage: python tools/qenc_fuse_ab.py [attribute]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(flag="fuse_ln", rounds=3, steps=30):
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    enc = HipBertEncoder.from_hf(BertModel(BertConfig(), add_pooling_layer=False).eval(), dev)
    res = {}
    for _ in range(rounds):
        for B in (8, 16, 32, 128):
            ids = torch.randint(1000, 30522, (B, 32), device=dev)
            mask = torch.ones((B, 32), dtype=torch.int64, device=dev)
            outs = {}
            for fuse in (False, True):
                setattr(enc, flag, fuse)
                outs[fuse] = enc(ids, mask).clone()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    enc.pool(enc(ids, mask), mask, "first")
                torch.cuda.synchronize()
                res.setdefault(f"b{B}_{'fused' if fuse else 'unfused'}", []).append(
                    round((time.perf_counter() - t0) / steps * 1e3, 4))
            res[f"b{B}_identical"] = bool(torch.equal(outs[False], outs[True]))
    print(json.dumps({"flag": flag, **{k: (sorted(v)[len(v) // 2] if isinstance(v, list) else v)
                                       for k, v in res.items()}}))


if __name__ == "__main__":
    main(*sys.argv[1:2])
