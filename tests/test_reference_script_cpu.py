"""CPU: the reference's own entry script ``run_random_sampling.py`` driven UNCHANGED through this
build's overlay (what ``python -m denseretrievaltoolkits_amd.run run_random_sampling.py ...`` does),
offline: a tiny BERT + tokenizer saved to a temp dir (--model_name_or_path), NQ-format jsonl splits
(--data_dir, the Tevatron/wikipedia-nq fields the reference's preprocessors read) and the
``wiki/corpus.json`` its CorpusDataset loads (--data_cache_dir).

Covered: HfArgumentParser over the reference's dataclasses, tokenizer + ``DRModel.build`` (the
overlay's), the reference's datasets / samplers / dataloaders on top of it, the overlay's ``Trainer``
constructor, and one collated training batch in the shape the HIP tower consumes.  Not covered
here: ``Trainer.train`` / ``evaluate`` themselves need the GPU (no CPU path exists); they are run by
the GPU suite (tests/test_trainer_gpu.py, tests/test_multirank_gpu.py).  Host adjustments, both
outside the build: the Trainer's device placement is stubbed (no GPU here), and the tokenizer gets
transformers 4.x's ``prepare_for_model`` (the reference's collator calls it; transformers 5.15, the
one installed, removed it).

Reads the reference from /root/reference (skipped where it is absent, e.g. on the GPU box).
Opt-in (DRT_RUN_REFERENCE_SCRIPT=1): the test executes the reference checkout's own Python in-process,
and that checkout is untrusted third-party content, so a default pytest run never imports it.
"""
import json
import os
import runpy
import sys

import pytest

REF = "/root/reference"
SCRIPT = os.path.join(REF, "run_random_sampling.py")

pytestmark = [
    pytest.mark.skipif(not os.path.exists(SCRIPT), reason="reference checkout not present"),
    pytest.mark.skipif(os.environ.get("DRT_RUN_REFERENCE_SCRIPT") != "1",
                       reason="runs untrusted reference code in-process: opt in with DRT_RUN_REFERENCE_SCRIPT=1"),
]

WORDS = ["paris", "france", "capital", "tower", "river", "seine", "london", "england", "what", "is", "the",
         "of", "city", "big", "bridge"]


def _assets(tmp):
    from transformers import BertConfig, BertModel, BertTokenizerFast
    vocab = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + WORDS
    mdir = os.path.join(tmp, "model")
    os.makedirs(mdir)
    with open(os.path.join(mdir, "vocab.txt"), "w") as f:
        f.write("\n".join(vocab) + "\n")
    BertTokenizerFast(os.path.join(mdir, "vocab.txt")).save_pretrained(mdir)
    cfg = BertConfig(vocab_size=len(vocab), hidden_size=64, num_hidden_layers=1, num_attention_heads=1,
                     intermediate_size=128, max_position_embeddings=64)
    BertModel(cfg).save_pretrained(mdir)
    ddir = os.path.join(tmp, "data")
    os.makedirs(ddir)
    rows = [{"query_id": str(i), "query": "what is the capital of france", "answers": ["paris"],
             "positive_passages": [{"docid": str(i), "title": "t", "text": WORDS[i] + " city"}],
             "negative_passages": [{"docid": str(i + 3), "title": "t", "text": WORDS[i + 3] + " river"}]}
            for i in range(8)]
    for split in ("train", "dev", "test"):
        with open(os.path.join(ddir, f"{split}.jsonl"), "w") as f:
            f.writelines(json.dumps(r) + "\n" for r in rows)
    cache = os.path.join(tmp, "cache")
    os.makedirs(os.path.join(cache, "wiki"))
    with open(os.path.join(cache, "wiki", "corpus.json"), "w") as f:
        f.writelines(json.dumps({"id": str(i), "title": "t", "text": w + " city paris"}) + "\n"
                     for i, w in enumerate(WORDS))
    return mdir, ddir, cache


def _prepare_for_model(self, ids, truncation=None, max_length=None, padding=False, return_attention_mask=False,
                       return_token_type_ids=False, **kw):
    """transformers 4.x PreTrainedTokenizerBase.prepare_for_model for one sequence, as the
    reference's collator calls it (truncate to max_length with the two special tokens, no padding)."""
    from transformers import BatchEncoding
    if max_length is not None:
        ids = list(ids)[: max(0, max_length - 2)]
    return BatchEncoding({"input_ids": [self.cls_token_id] + list(ids) + [self.sep_token_id]})


@pytest.fixture
def isolated_drt_modules():
    """The overlay registers DRT.* modules; drop whatever this test imported afterwards."""
    before = set(sys.modules)
    yield
    for name in set(sys.modules) - before:
        if name == "DRT" or name.startswith("DRT."):
            del sys.modules[name]


def test_run_random_sampling_script_through_overlay(tmp_path, monkeypatch, isolated_drt_modules):
    import torch
    for v in ("HF_HUB_OFFLINE", "TRANSFORMERS_OFFLINE", "HF_DATASETS_OFFLINE"):
        monkeypatch.setenv(v, "1")
    mdir, ddir, cache = _assets(str(tmp_path))
    monkeypatch.syspath_prepend(REF)
    from denseretrievaltoolkits_amd import drt_overlay
    drt_overlay.install()
    import DRT.model.biencoder as bi
    import DRT.trainer.trainer as tr
    from transformers import PreTrainedTokenizerBase
    assert tr.Trainer.__module__.startswith("denseretrievaltoolkits_amd")
    assert bi.DRModel.__module__.startswith("denseretrievaltoolkits_amd")

    got = {}

    def no_gpu_placement(self):   # Trainer._wrapper_model puts the model on the rank's GPU
        self.world, self.rank, self.local_rank = 1, 0, 0
        self.device = torch.device("cpu")

    monkeypatch.setattr(tr.Trainer, "_wrapper_model", no_gpu_placement)
    monkeypatch.setattr(tr.Trainer, "train", lambda self: got.setdefault("trainer", self))
    monkeypatch.setattr(PreTrainedTokenizerBase, "prepare_for_model", _prepare_for_model, raising=False)
    argv = ["run_random_sampling.py", "--train_batch_size", "4", "--eval_batch_size", "4", "--corpus_batch_size", "4",
            "--test_batch_size", "4", "--topk", "5,10", "--retrieve_num", "10",
            "--output_dir", str(tmp_path / "out"), "--model_name_or_path", mdir, "--dataset", "nq",
            "--data_dir", ddir, "--data_cache_dir", cache, "--train_n_passages", "2", "--q_max_len", "8",
            "--p_max_len", "16", "--max_epochs", "1", "--dataset_proc_num", "1", "--untie_encoder"]
    monkeypatch.setattr(sys, "argv", argv)
    mod = runpy.run_path(SCRIPT, run_name="drt_reference_script")   # not __main__: no NCCL init
    mod["main"]()

    t = got["trainer"]
    assert isinstance(t, tr.Trainer) and isinstance(t.model, bi.DRModel)
    assert t.training_args.topk == [5, 10] and t.training_args.retrieve_num == 10
    assert t.model.lm_q is not t.model.lm_p                       # --untie_encoder
    assert t.model.lm_q.config.hidden_size == 64                  # the saved tiny BERT
    assert t.corpus_dataloader is not None and t.eval_loader is not None and t.test_loader is not None
    # one collated training batch, in the layout DRModel.forward / the HIP tower take
    batch = next(iter(t.train_loader))
    q, p = batch[0], batch[1]
    assert q["input_ids"].shape[0] == 4 and q["input_ids"].shape[1] <= 8
    assert p["input_ids"].shape[0] == 4 * 2 and p["input_ids"].shape[1] <= 16
    assert (q["input_ids"][:, 0] == 2).all()                     # [CLS] first, as the collator builds it
