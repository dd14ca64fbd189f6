"""GPU: the HIP training tower (model/train_tower.py) against HF BertModel under
torch fp32 autograd on the same weights and inputs (dropout-free configuration): hidden states
and every parameter gradient, plus the dgrad-with-residual and GELU-forward pieces it adds."""
import numpy as np
import pytest

from oracle import bert_weights as bw

pytestmark = pytest.mark.gpu


def _bert(layers, seed, dev):
    import torch
    from transformers import BertModel
    torch.manual_seed(0)
    cfg = bw.bert_config(layers=layers)
    cfg.hidden_dropout_prob = 0.0
    cfg.attention_probs_dropout_prob = 0.0
    m = BertModel(cfg, add_pooling_layer=False)
    bw.init_model_(m, seed)
    return m.to(dev)


@pytest.mark.parametrize("layers,B,L", [(2, 4, 64), (1, 8, 128), (2, 6, 32)])
def test_tower_grads_vs_hf_autograd(dev, layers, B, L):
    import torch
    from denseretrievaltoolkits_amd.model.train_tower import train_hidden
    m_ref = _bert(layers, 11, dev).train()
    m_hip = _bert(layers, 11, dev).train()
    ids, mask = bw.token_batch(B, L, seed=L + B)
    ids_t, mask_t = torch.from_numpy(ids).to(dev), torch.from_numpy(mask).to(dev)
    g = torch.Generator(device=dev).manual_seed(5)
    R = torch.randn(B, L, 768, generator=g, device=dev)
    ref = m_ref(input_ids=ids_t, attention_mask=mask_t).last_hidden_state
    (ref * R).sum().backward()
    hid = train_hidden(m_hip, ids_t, mask_t)
    (hid * R).sum().backward()
    cos_h = torch.nn.functional.cosine_similarity(hid.flatten(), ref.detach().flatten(), dim=0).item()
    assert cos_h > 0.9999, cos_h
    worst, bad = [], []
    for (n, p_ref), (n2, p_hip) in zip(m_ref.named_parameters(), m_hip.named_parameters()):
        assert n == n2
        if p_ref.grad is None:
            assert p_hip.grad is None or float(p_hip.grad.abs().max()) == 0.0, n
            continue
        assert p_hip.grad is not None, n
        a, b = p_hip.grad.flatten().double(), p_ref.grad.flatten().double()
        nb = float(b.norm())
        if nb == 0.0:
            continue
        rel = float((a - b).norm()) / nb
        cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
        if n.endswith("attention.self.key.bias"):
            # softmax is invariant to a per-query constant, so d/d(key bias) is exactly 0; both sides
            # hold rounding noise -- require it small next to the value-bias gradient instead
            vb = dict(m_ref.named_parameters())[n.replace("key.bias", "value.bias")].grad.double().norm()
            if float(a.norm()) > 0.05 * float(vb):
                bad.append((n, float(a.norm()), float(vb)))
            continue
        worst.append((rel, cos, n))
        if not (cos > 0.995 and rel < 0.1):
            bad.append((n, cos, rel))
    worst.sort(reverse=True)
    print("worst relative gradient errors:", worst[:4])
    assert not bad, bad


def test_tower_rejects_dropout(dev):
    import torch
    from transformers import BertModel
    from denseretrievaltoolkits_amd.model.train_tower import train_hidden
    cfg = bw.bert_config(layers=1)
    cfg.hidden_dropout_prob = 0.1        # HF's default: the tower has no dropout masks yet
    m = BertModel(cfg, add_pooling_layer=False).to(dev)
    with pytest.raises(NotImplementedError):
        train_hidden(m, torch.ones((1, 8), dtype=torch.int64, device=dev), None)


def test_gelu_forward_vs_torch(dev):
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    x = (3 * torch.randn(100003, device=dev)).to(torch.bfloat16)
    y = torch.empty_like(x)
    _native.check(lib.drt_gelu_bf16(x.data_ptr(), x.numel(), y.data_ptr(), _native.stream_ptr(dev)), "gelu")
    ref = torch.nn.functional.gelu(x.float()).to(torch.bfloat16)
    assert float((y.float() - ref.float()).abs().max()) <= 2 ** -7 * float(ref.float().abs().max())
