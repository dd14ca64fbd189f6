#!/usr/bin/env python3
"""A/B of CU-masked streams for the encoder's two half-batch streams (HipBertEncoder._run_halves): each
half's kernels on its own half of the CUs (hipExtStreamCreateWithCUMask) instead of both halves sharing
every CU.  Times the passage tower (batch 512 x 128 tokens, BERT-base, random init) per mode, rounds
alternating.  usage: python tools/enc_cumask_ab.py [--modes none,even,split] [--rounds 3] [--steps 10]"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def masked_streams(dev, mode, ncu):
    import torch
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]
    words = (ncu + 31) // 32
    out = []
    for half in range(2):
        bits = [0] * words
        for cu in range(ncu):
            own = (cu % 2 == half) if mode == "even" else ((cu < ncu // 2) == (half == 0))
            if own:
                bits[cu // 32] |= 1 << (cu % 32)
        arr = (ctypes.c_uint32 * words)(*bits)
        s = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, arr)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
        out.append(torch.cuda.ExternalStream(s.value, device=dev))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="none,even,split")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, dev)
    del m
    g = torch.Generator(device=dev).manual_seed(1)
    ids = torch.randint(1000, 30522, (512, 128), generator=g, device=dev, dtype=torch.int64)
    ids[:, 0] = 101
    mask = torch.ones_like(ids)
    streams = {"none": None}
    for mode in a.modes.split(","):
        if mode != "none":
            streams[mode] = masked_streams(dev, mode, ncu)
    ref = None
    for rnd in range(a.rounds):
        for mode in a.modes.split(","):
            enc._streams = streams[mode]
            for _ in range(2):
                r = enc.pool(enc(ids, mask), mask, "first")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                r = enc.pool(enc(ids, mask), mask, "first")
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            r = r[0] if isinstance(r, (tuple, list)) else r
            if ref is None:
                ref = r.clone()
            print(json.dumps({"round": rnd, "mode": mode, "ms_per_batch": round(el / a.steps * 1e3, 3),
                              "passages_per_s": round(a.steps * 512 / el, 1),
                              "equal_to_first": bool(torch.equal(r, ref))}), flush=True)


if __name__ == "__main__":
    main()
