#!/usr/bin/env python3
"""Run bench.py's encoder-side legs one at a time with a progress line before and after each
(flushed), and optionally log every HipBertEncoder linear launch (shape, plan workspace, buffer
pointers) just before it reaches the C ABI -- so a run under `rocprofv3 --pmc ...` that dies shows
which leg, and which call, it died in.  Measurement support only (round-3 verdict: the PMC pass
segfaulted inside the HIP runtime under drt_linear_bf16_ws).

usage: python tools/pmc_legs.py [--legs encode,rerank,query,scores,train,recipe,evaluate] [--trace-linear]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", default="encode,rerank,query,scores,train,recipe,evaluate")
    ap.add_argument("--trace-linear", action="store_true")
    ap.add_argument("--c2-passages", type=int, default=200_000)
    ap.add_argument("--maps", default="", help="write /proc/self/maps here before each leg (to symbolise a "
                                               "crash's raw frame addresses offline: tools/symbolize_crash.py)")
    args = ap.parse_args()
    import faulthandler
    faulthandler.enable()
    import torch
    import bench_legs as bl
    from denseretrievaltoolkits_amd.model import encoder as enc_mod
    dev = torch.device("cuda", 0)
    ncall = [0]
    if args.trace_linear:
        orig_lin = enc_mod.HipBertEncoder._lin

        def traced(self, x, w, b, y, resid=None, gelu=False):
            ncall[0] += 1
            ws = getattr(self, "_ws", None)
            print(f"lin#{ncall[0]} x{tuple(x.shape)}:{x.dtype} w{tuple(w.shape)} y{tuple(y.shape)}:{y.dtype} "
                  f"gelu={gelu} resid={resid is not None} x=0x{x.data_ptr():x} y=0x{y.data_ptr():x} "
                  f"ws={'0x%x/%d' % (ws.data_ptr(), ws.numel() * 4) if ws is not None else None} "
                  f"stream=0x{int(self.stream or 0):x}", file=sys.stderr, flush=True)
            return orig_lin(self, x, w, b, y, resid=resid, gelu=gelu)
        enc_mod.HipBertEncoder._lin = traced
    legs = {
        "encode": lambda: bl.run(dev, steps=3, warmup=1),
        "rerank": lambda: bl.run_rerank(dev, steps=1, warmup=1),
        "query": lambda: bl.run_query_encode(dev, steps=5, warmup=1),
        "scores": lambda: bl.run_train_scores(dev, steps=3, warmup=1),
        "train": lambda: bl.run_train_step(dev, steps=1, warmup=1),
        "recipe": lambda: bl.run_train_step(dev, bq=128, n=8, p_len=156, steps=1, warmup=1),
        "evaluate": lambda: bl.run_evaluate_c2(dev, n_passages=args.c2_passages),
    }
    torch.zeros(1, device=dev)   # the runtime (and a profiler's hooks) loaded before the first map dump
    for name in args.legs.split(","):
        if args.maps:
            with open("/proc/self/maps") as src, open(args.maps, "w") as dst:
                dst.write(src.read())
        print(f"LEG {name} start (linear calls so far {ncall[0]})", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        legs[name]()
        torch.cuda.synchronize()
        print(f"LEG {name} done {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
