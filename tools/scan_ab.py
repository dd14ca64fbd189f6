#!/usr/bin/env python3
"""Interleaved A/B of filter-scan variants on the bench workload (10M x 768 bf16, Qb 128, k 1000).

One process, one corpus; every round times each variant for --steps launches (HIP events
around the filter scan, drt_profile_*), so box-to-box DVFS differences cancel.  Variants that
compute real results must return ids identical to variant 0.
usage: python tools/scan_ab.py [--variants 0,12,13] [--rounds 3] [--steps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,12,13,14,15,17")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--qb", type=int, default=128)
    ap.add_argument("--k", type=int, default=1000)
    args = ap.parse_args()
    import torch
    from bench import gen_shard
    from denseretrievaltoolkits_amd import _native, kernels
    dev = torch.device("cuda", 0)
    lib = _native.load()
    shard, lo, hi = gen_shard(args.n, 1, 0, 768, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(5678)
    qs = torch.randn((args.steps, args.qb, 768), generator=g, device=dev).to(torch.bfloat16)
    variants = [int(v) for v in args.variants.split(",")]
    ref = {}
    times = {v: [] for v in variants}
    for rnd in range(args.rounds):
        for v in variants:
            _native.check(lib.drt_scan_variant(v), "variant")
            kernels.ip_topk(qs[0], shard, args.k, resolve=False)  # warm
            torch.cuda.synchronize()
            lib.drt_profile_enable(_native.PROF_SCAN, 1)
            outs = [kernels.ip_topk(qs[j], shard, args.k, resolve=False) for j in range(args.steps)]
            torch.cuda.synchronize()
            lib.drt_profile_enable(_native.PROF_SCAN, 0)
            tot = _native.ctypes.c_double(0.0)
            cnt = _native.c_i64(0)
            lib.drt_profile_read(_native.PROF_SCAN, _native.ctypes.byref(tot), _native.ctypes.byref(cnt))
            times[v].append(tot.value / max(1, cnt.value))
            if rnd == 0:
                ids = torch.stack([o[1] for o in outs]).cpu()
                if v == variants[0]:
                    ref["ids"] = ids
                elif v >= 12:
                    same = bool(torch.equal(ids, ref["ids"]))
                    print(f"variant {v}: ids identical to variant {variants[0]}: {same}", flush=True)
            print(f"round {rnd} variant {v}: {times[v][-1]:.4f} ms", flush=True)
    _native.check(lib.drt_scan_variant(0), "variant")
    alg = args.n * 768 * 2 + args.qb * 768 * 2 + args.qb * args.k * 12
    res = {v: {"ms_min": min(t), "ms_mean": sum(t) / len(t), "tbps_best": alg / min(t) / 1e9}
           for v, t in times.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
