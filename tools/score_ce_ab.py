#!/usr/bin/env python3
"""A/B of the fused score + CE (bench leg train_scores: batch 512, d 768, n = 2 / 8) for one library
variant (DRT_LIB=<variants/libdrt_hip.X.so>, tools/build_variant.sh), plus its loss / grads against torch
fp32 autograd.  usage: DRT_LIB=... python tools/score_ce_ab.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_legs  # noqa: E402
from denseretrievaltoolkits_amd.score_ce import score_ce  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    q = torch.randn((512, 768), generator=g, device=dev).requires_grad_(True)
    p = torch.randn((4096, 768), generator=g, device=dev).requires_grad_(True)
    loss, _ = score_ce(q, p, 8, 1.0)
    loss.backward()
    q2, p2 = q.detach().clone().requires_grad_(True), p.detach().clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(q2 @ p2.T, torch.arange(512, device=dev) * 8)
    ref.backward()
    err = {"loss": abs(loss.item() - ref.item()), "dq": float((q.grad - q2.grad).abs().max()),
           "dp": float((p.grad - p2.grad).abs().max())}
    res = bench_legs.run_train_scores(dev)
    print(json.dumps({"lib": os.path.basename(os.environ.get("DRT_LIB", "product")), "err": err,
                      "n2": {k: res["n2"][k] for k in ("hip_ms", "hip_graph_ms", "torch_graph_ms")},
                      "n8": {k: res["n8"][k] for k in ("hip_ms", "hip_graph_ms", "torch_graph_ms")}}), flush=True)


if __name__ == "__main__":
    main()
