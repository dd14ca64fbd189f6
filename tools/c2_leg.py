#!/usr/bin/env python3
"""bench_legs.run_evaluate_c2 alone (config C2 through Trainer.evaluate), `--rounds` times in one process:
the stage timers, device-only times and the certification counters, one JSON line per round.
usage: python tools/c2_leg.py [--passages 1000000] [--rounds 2]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passages", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import bench_legs as bl
    dev = torch.device("cuda", 0)
    for rnd in range(args.rounds):
        d = bl.run_evaluate_c2(dev, n_passages=args.passages)
        print(json.dumps({"round": rnd, **{k: d[k] for k in ("stages_s", "device_only", "queries_per_s_end_to_end",
                                                             "passages_per_s", "recall@1000")}}), flush=True)


if __name__ == "__main__":
    main()
