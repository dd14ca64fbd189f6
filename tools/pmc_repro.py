#!/usr/bin/env python3
"""Smallest steps towards the rocprofv3 --pmc abort seen in the evaluate leg (SIGSEGV in a memcpy
under THCPEvent_wait / hipLaunchKernel, no DRT frame below it): each step prints before it runs, so
the last line names the HIP operation the profiler fails on.  Torch ops only (no DRT kernels)."""
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
    say("done")


if __name__ == "__main__":
    main()
