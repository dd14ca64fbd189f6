#!/usr/bin/env python3
"""Smallest steps towards the rocprofv3 --pmc abort seen in the evaluate leg (SIGSEGV in a memcpy
under THCPEvent_wait / hipLaunchKernel, no DRT frame below it): each step prints before it runs, so
the last line names the HIP operation the profiler fails on.  Torch ops only (no DRT kernels).
usage: python tools/pmc_repro.py [N [nocopy]]   (N > 0: step 9, N tiny kernels on a side stream; nocopy:
without the pinned H2D copies)"""
import sys

import torch


def say(msg):
    print(msg, file=sys.stderr, flush=True)


def main():
    dev = torch.device("cuda", 0)
    x = torch.randn(1 << 20, device=dev)
    say("1 kernels on the default stream")
    for _ in range(10):
        x = x * 1.0001 + 1.0
    torch.cuda.synchronize()
    say("2 second stream + wait_stream")
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        y = x * 2.0
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    say("3 event record + event wait")
    ev = torch.cuda.Event()
    ev.record(s)
    ev.wait(torch.cuda.current_stream(dev))
    z = y + 1.0
    torch.cuda.synchronize()
    say("4 pinned non-blocking D2H + event synchronize")
    h = torch.empty(z.shape, dtype=z.dtype, pin_memory=True)
    h.copy_(z, non_blocking=True)
    e2 = torch.cuda.Event()
    e2.record()
    e2.synchronize()
    say("5 many streams (more than GPU_MAX_HW_QUEUES)")
    ss = [torch.cuda.Stream(dev) for _ in range(8)]
    for st in ss:
        with torch.cuda.stream(st):
            _ = x + 3.0
    torch.cuda.synchronize()
    say("6 event wait across fresh streams")
    for st in ss:
        e = torch.cuda.Event()
        e.record(st)
        e.wait(torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    say("7 pinned H2D non-blocking on a side stream, event wait on the current stream")
    hp = torch.randn(1 << 22).pin_memory()
    s2 = torch.cuda.Stream(dev)
    with torch.cuda.stream(s2):
        dv = hp.to(dev, non_blocking=True)
        e3 = torch.cuda.Event()
        e3.record(s2)
    e3.wait(torch.cuda.current_stream(dev))
    _ = dv * 2.0
    torch.cuda.synchronize()
    say("8 the same, many times")
    for _ in range(50):
        with torch.cuda.stream(s2):
            dv = hp.to(dev, non_blocking=True)
            e4 = torch.cuda.Event()
            e4.record(s2)
        e4.wait(torch.cuda.current_stream(dev))
        _ = dv * 2.0
    torch.cuda.synchronize()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    copies = "nocopy" not in sys.argv[2:]
    if n:
        # the evaluate leg dies after ~9k encoder linears (tens of thousands of dispatches): the same
        # number of tiny kernels on one side stream, a pinned H2D copy every 64 of them
        say(f"9 {n} kernels on a side stream with periodic pinned H2D copies")
        s3 = torch.cuda.Stream(dev)
        hb = torch.randint(0, 30000, (256, 128), dtype=torch.int64).pin_memory()
        with torch.cuda.stream(s3):
            acc = torch.zeros(256, 128, dtype=torch.int64, device=dev)
            for j in range(n):
                if j % 64 == 0 and copies:
                    acc += hb.to(dev, non_blocking=True)
                else:
                    acc.add_(1)
                if j % 5000 == 0:
                    say(f"  kernel {j}")
        torch.cuda.synchronize()
    say("done")


if __name__ == "__main__":
    main()
