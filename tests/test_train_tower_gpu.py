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


@pytest.mark.parametrize("layers,B,L", [(2, 4, 64), (1, 8, 128), (2, 6, 32), (1, 4, 156)])
def test_tower_grads_vs_hf_autograd(dev, layers, B, L):
    _grads_vs_hf(dev, layers, B, L, types=False)


@pytest.mark.parametrize("layers,B,L", [(1, 6, 64), (2, 4, 156), (1, 3, 256), (1, 2, 512)])
def test_tower_grads_with_token_types_vs_hf_autograd(dev, layers, B, L):
    """token_type_ids given (segment A = 0, segment B = 1, as a pair encoder would): the type
    embeddings enter the forward and the type-row gradients come from per-type column sums."""
    _grads_vs_hf(dev, layers, B, L, types=True)


def _grads_vs_hf(dev, layers, B, L, types):
    import torch
    from denseretrievaltoolkits_amd.model.train_tower import train_hidden
    m_ref = _bert(layers, 11, dev).train()
    m_hip = _bert(layers, 11, dev).train()
    ids, mask = bw.token_batch(B, L, seed=L + B)
    ids_t, mask_t = torch.from_numpy(ids).to(dev), torch.from_numpy(mask).to(dev)
    tt = None
    if types:
        rng = np.random.default_rng(L)
        cut = rng.integers(1, L, size=(B, 1))
        tt = torch.from_numpy((np.arange(L)[None, :] >= cut).astype(np.int64)).to(dev)
    g = torch.Generator(device=dev).manual_seed(5)
    R = torch.randn(B, L, 768, generator=g, device=dev)
    ref = m_ref(input_ids=ids_t, attention_mask=mask_t, token_type_ids=tt).last_hidden_state
    (ref * R).sum().backward()
    hid = train_hidden(m_hip, ids_t, mask_t, token_type_ids=tt)
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


def test_tower_rejects_unsupported(dev):
    import torch
    from transformers import BertModel
    from denseretrievaltoolkits_amd.model.train_tower import train_hidden
    m = BertModel(bw.bert_config(layers=1), add_pooling_layer=False).to(dev)
    with pytest.raises(ValueError):                      # past max_position_embeddings
        train_hidden(m, torch.ones((1, 513), dtype=torch.int64, device=dev), None)


def test_gelu_forward_vs_torch(dev):
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    x = (3 * torch.randn(100003, device=dev)).to(torch.bfloat16)
    y = torch.empty_like(x)
    _native.check(lib.drt_gelu_bf16(x.data_ptr(), x.numel(), y.data_ptr(), _native.stream_ptr(dev)), "gelu")
    ref = torch.nn.functional.gelu(x.float()).to(torch.bfloat16)
    assert float((y.float() - ref.float()).abs().max()) <= 2 ** -7 * float(ref.float().abs().max())


# ---- dropout: torch restatement of csrc/drt_common.h drop_hash24 (test-side mask generator)
_C1, _C2, _C3 = 0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB
_M64 = (1 << 64) - 1


def _s64(c):
    c &= _M64
    return c - (1 << 64) if c >= (1 << 63) else c


def _hash24_py(seed, site, idx):
    x = (idx * _C1 + seed + site * _C2) & _M64
    x ^= x >> 31
    x = (x * _C3) & _M64
    x ^= x >> 29
    return x >> 40


def _keep_torch(seed, site, idx, p):
    import torch
    x = idx * _s64(_C1) + _s64(seed + site * _C2)
    x = x ^ ((x >> 31) & ((1 << 33) - 1))
    x = x * _s64(_C3)
    x = x ^ ((x >> 29) & ((1 << 35) - 1))
    h = (x >> 40) & ((1 << 24) - 1)
    return h >= int(np.float32(p) * np.float32(16777216.0))


# attention-probability dropout (csrc/drt_common.h attn_row_key / attn_mix): two keep decisions per
# 32-bit hash of (row key, key pair), 16-bit thresholds
_G32, _F1, _F2 = 0x9E3779B9, 0x85EBCA6B, 0xC2B2AE35
_M32 = (1 << 32) - 1


def _attn_keep_py(seed, site, row, key, p):
    x = (row * _C1 + seed + site * _C2) & _M64
    x ^= x >> 31
    x = (x * _C3) & _M64
    x ^= x >> 29
    h = ((x >> 32) + (key >> 1) * _G32) & _M32
    h ^= h >> 16
    h = (h * _F1) & _M32
    h ^= h >> 13
    h = (h * _F2) & _M32
    h ^= h >> 16
    half = (h >> 16) if key & 1 else (h & 0xFFFF)
    return half >= int(np.float32(p) * np.float32(65536.0))


def _attn_keep_torch(seed, site, B, heads, L, p, device):
    """[B][heads][L query][L key] keep mask of the attention-probability dropout."""
    import torch
    row = torch.arange(B * heads * L, device=device, dtype=torch.int64)
    x = row * _s64(_C1) + _s64(seed + site * _C2)
    x = x ^ ((x >> 31) & ((1 << 33) - 1))
    x = x * _s64(_C3)
    x = x ^ ((x >> 29) & ((1 << 35) - 1))
    rk = (x >> 32) & _M32
    key = torch.arange(L, device=device, dtype=torch.int64)
    h = (rk[:, None] + (key >> 1)[None, :] * _G32) & _M32
    h = h ^ (h >> 16)
    h = (h * _F1) & _M32
    h = h ^ (h >> 13)
    h = (h * _F2) & _M32
    h = h ^ (h >> 16)
    half = torch.where((key & 1).bool()[None, :], h >> 16, h & 0xFFFF)
    return (half >= int(np.float32(p) * np.float32(65536.0))).view(B, heads, L, L)


def test_dropout_kernel_mask_matches_restatement(dev):
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    n = 1 << 20
    y = torch.randn(n, device=dev).to(torch.bfloat16)
    r = torch.randn(n, device=dev).to(torch.bfloat16)
    out = torch.empty_like(y)
    seed, site, p = 987654321, 5, 0.1
    _native.check(lib.drt_dropout_add_bf16(y.data_ptr(), r.data_ptr(), n, p, seed, site, out.data_ptr(),
                                           _native.stream_ptr(dev)), "dropout")
    keep = _keep_torch(seed, site, torch.arange(n, device=dev, dtype=torch.int64), p)
    ref = (torch.where(keep, y.float() / (1 - p), torch.zeros_like(y.float())) + r.float()).to(torch.bfloat16)
    assert torch.equal(out[~keep], r[~keep])                  # dropped: exactly the residual -> same mask
    err = (out.float() - ref.float()).abs()
    scale = y.float().abs() / (1 - p) + r.float().abs()          # kept: one bf16 rounding of the operands
    assert bool((err <= scale * 2.0 ** -7).all())
    assert abs(float(keep.float().mean()) - 0.9) < 0.002


def _ref_forward_with_masks(m, ids, mask, ph, pa, seed):
    """Functional fp32 BERT forward (modeling_bert.py semantics) with the kernels' dropout masks."""
    import torch
    import torch.nn.functional as F
    from denseretrievaltoolkits_amd.model.train_tower import dropout_sites
    cfg = m.config
    B, L = ids.shape
    H, nh = cfg.hidden_size, cfg.num_attention_heads
    dh = H // nh
    eps = cfg.layer_norm_eps
    dev = ids.device
    flat = torch.arange(B * L * H, device=dev, dtype=torch.int64).view(B, L, H)

    def drop(x, site, p, idx):
        return torch.where(_keep_torch(seed, site, idx, p), x / (1 - p), torch.zeros_like(x)) if p > 0 else x

    def drop_probs(x, site, p):
        keep = _attn_keep_torch(seed, site, B, nh, L, p, dev)
        return torch.where(keep, x / (1 - p), torch.zeros_like(x)) if p > 0 else x

    e = m.embeddings
    x = e.word_embeddings(ids) + e.token_type_embeddings(torch.zeros_like(ids)) + \
        e.position_embeddings(torch.arange(L, device=dev))[None]
    x = drop(F.layer_norm(x, (H,), e.LayerNorm.weight, e.LayerNorm.bias, eps), 0, ph, flat)
    bias = (1 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
    for i, layer in enumerate(m.encoder.layer):
        s_att, s1, s2 = dropout_sites(i)
        sa = layer.attention.self
        q = sa.query(x).view(B, L, nh, dh).transpose(1, 2)
        k = sa.key(x).view(B, L, nh, dh).transpose(1, 2)
        v = sa.value(x).view(B, L, nh, dh).transpose(1, 2)
        probs = torch.softmax(q @ k.transpose(-1, -2) / dh ** 0.5 + bias, -1)
        ctx = (drop_probs(probs, s_att, pa) @ v).transpose(1, 2).reshape(B, L, H)
        ao = layer.attention.output
        x1 = F.layer_norm(drop(ao.dense(ctx), s1, ph, flat) + x, (H,), ao.LayerNorm.weight, ao.LayerNorm.bias, eps)
        f = F.gelu(layer.intermediate.dense(x1))
        o = layer.output
        x = F.layer_norm(drop(o.dense(f), s2, ph, flat) + x1, (H,), o.LayerNorm.weight, o.LayerNorm.bias, eps)
    return x


@pytest.mark.parametrize("layers,B,L", [(2, 4, 64), (1, 6, 128), (1, 3, 156), (1, 2, 384)])
def test_tower_with_dropout_vs_masked_fp32_reference(dev, layers, B, L):
    """Train-mode tower with HF's default dropout (0.1 / 0.1) against a functional fp32 BERT under
    autograd that applies the SAME hash masks: hidden states and every parameter gradient."""
    import torch
    from denseretrievaltoolkits_amd.model.train_tower import train_hidden
    m_ref = _bert(layers, 13, dev).train()
    m_hip = _bert(layers, 13, dev).train()
    for m in (m_ref, m_hip):
        m.config.hidden_dropout_prob = 0.1
        m.config.attention_probs_dropout_prob = 0.1
    ids, mask = bw.token_batch(B, L, seed=3 * L + B)
    ids_t, mask_t = torch.from_numpy(ids).to(dev), torch.from_numpy(mask).to(dev)
    seed = 24680
    R = torch.randn(B, L, 768, generator=torch.Generator(device=dev).manual_seed(9), device=dev)
    ref = _ref_forward_with_masks(m_ref, ids_t, mask_t, 0.1, 0.1, seed)
    (ref * R).sum().backward()
    hid = train_hidden(m_hip, ids_t, mask_t, seed=seed)
    (hid * R).sum().backward()
    cos_h = torch.nn.functional.cosine_similarity(hid.flatten(), ref.detach().flatten(), dim=0).item()
    assert cos_h > 0.9999, cos_h
    bad = []
    for (n, p_ref), (_, p_hip) in zip(m_ref.named_parameters(), m_hip.named_parameters()):
        if p_ref.grad is None or n.endswith("key.bias") or float(p_ref.grad.norm()) == 0.0:
            continue
        a, b = p_hip.grad.flatten().double(), p_ref.grad.flatten().double()
        cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
        rel = float((a - b).norm() / b.norm())
        if not (cos > 0.995 and rel < 0.1):
            bad.append((n, cos, rel))
    assert not bad, bad
