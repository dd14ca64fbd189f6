#!/usr/bin/env python3
"""Where the host time of Trainer.evaluate's query stage goes (bench evaluate_c2 at a smaller
corpus): cProfile of one evaluation after a warm-up one, top functions by cumulative and by own
time.  usage: python tools/c2_host_prof.py [--passages 200000] [--queries 10000]"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passages", type=int, default=200_000)
    ap.add_argument("--queries", type=int, default=10_000)
    args = ap.parse_args()
    import torch
    from types import SimpleNamespace
    from transformers import BertConfig, BertModel
    import bench_legs as bl
    from denseretrievaltoolkits_amd.model.biencoder import DRModel
    from denseretrievaltoolkits_amd.trainer.trainer import Trainer
    torch.manual_seed(0)
    lm = BertModel(BertConfig(), add_pooling_layer=False).eval()
    model = DRModel(lm_q=lm, lm_p=lm, pooling="first")
    targs = SimpleNamespace(loss_fn="SimpleContrastiveLoss", learning_rate=1e-5, optimizer="adamw",
                            topk="1,5,20,100,1000", retrieve_num=1000, retrieve_dir="", cache_train_dir="",
                            encode_corpus_dir="", index_order_dir="", max_epochs=0, save_per_train=1,
                            eval_per_train=1)
    corpus = bl._SyntheticCorpus(args.passages)
    cl = bl._Loader(4 * 512, 512, 128, 11, dataset=corpus)
    ql = bl._Loader(args.queries, 128, 32, 12, queries=True)
    tr = Trainer(targs, model, corpus_dataloader=cl, eval_loader=ql)
    tr.evaluate(ql, 0)
    tr.corpus_dataloader = bl._Loader(args.passages, 512, 128, 11, dataset=corpus)
    tr.profile_eval = True
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    tr.evaluate(ql, 1)
    torch.cuda.synchronize()
    pr.disable()
    print(f"evaluate {time.perf_counter() - t0:.2f} s; stages {tr.last_eval_timing}", flush=True)
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(28)
        print(s.getvalue()[-6000:], flush=True)


if __name__ == "__main__":
    main()
