#!/usr/bin/env python3
"""Symbolise the raw frame addresses of a crash log ("@ 0x7f... (unknown)" lines of the glog-style
stack a rocprofv3 tool prints) against a /proc/<pid>/maps dump of the same process (tools/pmc_legs.py
--maps): each address -> (library, file offset) -> llvm-symbolizer on that library (the libraries of this
image are the same files as on the GPU box).
usage: python tools/symbolize_crash.py <crash.log> <maps.txt>"""
import re
import subprocess
import sys


def main(log, maps):
    regions = []
    for line in open(maps):
        f = line.split()
        if len(f) < 6:
            continue
        a, b = (int(x, 16) for x in f[0].split("-"))
        regions.append((a, b, int(f[2], 16), f[5]))
    sym = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"
    for line in open(log):
        m = re.search(r"@\s+0x([0-9a-f]+)", line)
        if not m:
            continue
        addr = int(m.group(1), 16)
        hit = [(a, b, off, path) for a, b, off, path in regions if a <= addr < b]
        if not hit:
            print(f"0x{addr:x}  ?  {line.strip()}")
            continue
        a, b, off, path = hit[0]
        foff = addr - a + off
        try:
            out = subprocess.run([sym, "--obj", path, "--relative-address", hex(foff)], capture_output=True,
                                 text=True, timeout=30).stdout.split("\n")[0]
        except Exception as e:   # noqa: BLE001 (tooling)
            out = f"<{e}>"
        print(f"0x{addr:x}  {path}+0x{foff:x}  {out}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
