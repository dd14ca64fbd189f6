"""A/B: pipelined inference attention (one round of work-groups looping over (sequence, head) units,
next unit's loads under the current unit's work) vs one unit per work-group (drt_attention_pipe).

Kernel level: the encode leg's half-batch launch (256 x 128 tokens x 12 heads) and the query tower's
(128 x 32), all-ones and ragged masks; ctx bit-identical between the forms; HIP-event time per launch,
interleaved rounds.  Encode level: HipBertEncoder passages/s at 512 x 128 with each form."""
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(rounds=5, reps=50):
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    dev = torch.device("cuda", 0)
    stream = _native.stream_ptr(dev)
    heads, dh = 12, 64
    H = heads * dh
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    res = {}
    for (B, L, ragged) in ((256, 128, False), (256, 128, True), (128, 32, False), (64, 100, True)):
        qkv = (torch.randn((B * L, 3 * H), generator=g, device=dev) * 2).to(torch.bfloat16)
        mask = torch.ones((B, L), dtype=torch.int64, device=dev)
        if ragged:
            lens = torch.randint(L // 4, L + 1, (B,), generator=g, device=dev)
            mask = (torch.arange(L, device=dev)[None, :] < lens[:, None]).to(torch.int64)
        outs = {}
        times = {0: [], 1: []}
        scale = 1.0 / math.sqrt(dh)

        def run(on, ctx):
            lib.drt_attention_pipe(on)
            _native.check(lib.drt_attention_bf16(qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), B, L, heads, dh,
                                                 scale, stream), "attn")

        for on in (0, 1):
            ctx = torch.full((B * L, H), float("nan"), dtype=torch.bfloat16, device=dev)
            run(on, ctx)
            torch.cuda.synchronize()
            outs[on] = ctx
        for _ in range(rounds):
            for on in (0, 1):
                ctx = outs[on]
                run(on, ctx)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    run(on, ctx)
                e1.record()
                torch.cuda.synchronize()
                times[on].append(e0.elapsed_time(e1) * 1000 / reps)
        nbytes = B * L * 3 * H * 2 + B * L * H * 2
        key = f"B{B}_L{L}{'_ragged' if ragged else ''}"
        med = {on: sorted(v)[len(v) // 2] for on, v in times.items()}
        res[key] = {"one_unit_us": round(med[0], 2), "pipe_us": round(med[1], 2),
                    "pipe_over_one": round(med[1] / med[0], 3),
                    "pipe_hbm_frac": round(nbytes / (med[1] * 1e-6) / 8e12, 3),
                    "one_unit_hbm_frac": round(nbytes / (med[0] * 1e-6) / 8e12, 3),
                    "bit_identical": bool(torch.equal(outs[0], outs[1])),
                    "rounds_us": {str(k): [round(x, 2) for x in v] for k, v in times.items()}}
        print(json.dumps({key: res[key]}), flush=True)
    lib.drt_attention_pipe(1)

    # encode level
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, dev)
    del m
    B, L = 512, 128
    ids = torch.randint(1000, 30522, (B, L), device=dev)
    mask = torch.ones((B, L), dtype=torch.int64, device=dev)
    ref = {}
    pps = {0: [], 1: []}
    for _ in range(3):
        for on in (0, 1):
            lib.drt_attention_pipe(on)
            out = enc(ids, mask)
            torch.cuda.synchronize()
            ref.setdefault(on, out.clone())
            t0 = time.perf_counter()
            for _ in range(8):
                enc.pool(enc(ids, mask), mask, "first")
            torch.cuda.synchronize()
            pps[on].append(round(8 * B / (time.perf_counter() - t0), 1))
    lib.drt_attention_pipe(1)
    res["encode_512x128"] = {"one_unit": pps[0], "pipe": pps[1], "bit_identical": bool(torch.equal(ref[0], ref[1]))}
    print(json.dumps({"encode_512x128": res["encode_512x128"]}), flush=True)


if __name__ == "__main__":
    main()
