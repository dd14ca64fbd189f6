"""CPU: a ``feature`` other than ``last_hidden_state`` (reference DRT/arguments.py:34-37, read in
DRT/model/biencoder.py:137-138) takes the HF module in BOTH grad modes, with the reason logged, so
the no-grad (inference) and autograd encodes agree.  The HIP towers only serve last_hidden_state."""
import logging
from types import SimpleNamespace

import torch
from torch import nn

from denseretrievaltoolkits_amd.model import biencoder
from denseretrievaltoolkits_amd.model.biencoder import DRModel


class _TwoFeatures(nn.Module):
    """Stands in for an HF model whose output carries a second per-token feature."""

    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(16, 8)

    def forward(self, input_ids=None, attention_mask=None, return_dict=True, **kw):
        h = self.emb(input_ids)
        return SimpleNamespace(last_hidden_state=h, alt_feature=2.0 * h + 1.0)


def test_non_default_feature_agrees_across_grad_modes(monkeypatch, caplog):
    torch.manual_seed(0)
    lm = _TwoFeatures()
    m = DRModel(lm_q=lm, lm_p=lm, feature="alt_feature", pooling="mean")
    # pretend the tower sits on the GPU: the inference branch must still not take the HIP encoder
    monkeypatch.setattr(m, "_use_hip", lambda model: True)
    monkeypatch.setattr(m, "_hip_encoder", lambda model: (_ for _ in ()).throw(AssertionError("HIP encoder")))
    monkeypatch.setattr(biencoder, "_FALLBACK_LOGGED", set())
    items = {"input_ids": torch.tensor([[1, 2, 3, 0], [4, 5, 0, 0]]),
             "attention_mask": torch.tensor([[1, 1, 1, 0], [1, 1, 0, 0]])}
    want = lm(**items).alt_feature
    want = (want * items["attention_mask"][..., None]).sum(1) / items["attention_mask"].sum(1, keepdim=True)
    with caplog.at_level(logging.WARNING, logger=biencoder.__name__):
        with torch.no_grad():
            _, r_inf = m.encode_query(items)
        _, r_grad = m.encode_query(items)
    assert torch.allclose(r_inf, want.detach(), atol=1e-6)
    assert torch.equal(r_inf, r_grad.detach())
    assert r_grad.requires_grad
    assert "feature 'alt_feature'" in caplog.text
