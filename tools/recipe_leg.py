#!/usr/bin/env python3
"""The bench's train_step_recipe leg alone (run.sh shapes: batch 128, n 8, p_len 156), HIP tower
only unless --all: for timing and kernel traces.  usage: python tools/recipe_leg.py [--all] [--steps 3]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--p-len", type=int, default=156)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--bq", type=int, default=128)
    args = ap.parse_args()
    import bench_legs as bl
    dev = torch.device("cuda", 0)
    if args.all:
        print(json.dumps(bl.run_train_step(dev, bq=args.bq, n=args.n, p_len=args.p_len, steps=args.steps, warmup=1)))
        return
    from types import SimpleNamespace
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.biencoder import DRModel
    torch.manual_seed(0)
    lm = BertModel(BertConfig(), add_pooling_layer=False).to(dev).train()
    m = DRModel(lm_q=lm, lm_p=lm, pooling="first", data_args=SimpleNamespace(train_n_passages=args.n),
                train_args=SimpleNamespace(negatives_x_device=False)).train()
    g = torch.Generator(device=dev)
    g.manual_seed(6)

    def batch(b, L):
        ids = torch.randint(1000, 30522, (b, L), generator=g, device=dev, dtype=torch.int64)
        return {"input_ids": ids, "attention_mask": torch.ones((b, L), dtype=torch.int64, device=dev)}

    qry, psg = batch(args.bq, 32), batch(args.bq * args.n, args.p_len)

    def step():
        lm.zero_grad(set_to_none=True)
        m(query=qry, passage=psg).loss.backward()

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    print(json.dumps({"hip_ms": round((time.perf_counter() - t0) / args.steps * 1e3, 2), "p_len": args.p_len,
                      "n": args.n, "bq": args.bq}), flush=True)


if __name__ == "__main__":
    main()
