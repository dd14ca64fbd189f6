#!/usr/bin/env python3
"""C2 query stage A/B (bench_legs.run_evaluate_c2 at a given corpus size): Trainer.evaluate's stage
timers -- results wait (host blocked on search results), match issue / finish -- for the default
window order and EAGER_WINDOW_SEARCH.  usage: python tools/c2_ab.py [--passages 1000000] [--rounds 2]"""
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
    from denseretrievaltoolkits_amd.trainer.trainer import Trainer
    dev = torch.device("cuda", 0)
    for rnd in range(args.rounds):
        for eager in (False, True):
            Trainer.EAGER_WINDOW_SEARCH = eager
            d = bl.run_evaluate_c2(dev, n_passages=args.passages)
            print(json.dumps({"round": rnd, "eager": eager, "stages_s": {k: round(v, 4) for k, v in d["stages_s"].items()},
                              "device_only": d["device_only"], "qps_e2e": d["queries_per_s_end_to_end"]}), flush=True)


if __name__ == "__main__":
    main()
