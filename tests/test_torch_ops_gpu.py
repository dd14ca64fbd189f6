"""GPU: the torch.ops.drt custom operators (csrc/torch_ops.cpp over include/drt.h).

torch.ops.drt.ip_topk returns the oracle's ids and scores bit for bit (integer-valued inputs,
exact in fp32; reference semantics: BaseFaissIPRetriever.search, DRT/evaluator/index.py:31-33),
and torch.library.opcheck validates schema, fake implementation, autograd registration and
AOT dispatch of every functional operator."""
import numpy as np
import pytest

from helpers import int_bf16, to_dev_bf16
from oracle import search_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def drt(dev):
    from denseretrievaltoolkits_amd import ops
    return ops.load()


def test_ip_topk_op_bit_exact(dev, drt):
    import torch
    rng = np.random.default_rng(5)
    q = int_bf16(rng, (40, 768), -4, 4)
    p = int_bf16(rng, (60000, 768), -4, 4)
    s, i, st = drt.ip_topk(to_dev_bf16(q, dev), to_dev_bf16(p, dev), 1000, 7)
    torch.cuda.synchronize()
    es, ei = orc.ip_topk(q, p, 1000, id_offset=7)
    assert (st.cpu().numpy() == 0).all()
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    np.testing.assert_array_equal(s.cpu().numpy(), es)


def test_ip_topk_resolve_op(dev, drt):
    """Status forced to 1 for some queries: the op rescans them exactly and clears the status."""
    import torch
    rng = np.random.default_rng(6)
    q = int_bf16(rng, (9, 256), -4, 4)
    p = int_bf16(rng, (30000, 256), -4, 4)
    qd, pd = to_dev_bf16(q, dev), to_dev_bf16(p, dev)
    s, i, st = drt.ip_topk(qd, pd, 100, 0)
    s[[1, 4]] = 0.0
    i[[1, 4]] = 0
    st[[1, 4]] = 1
    n = drt.ip_topk_resolve(qd, pd, 100, 0, s, i, st)
    assert n == 2 and (st.cpu().numpy() == 0).all()
    es, ei = orc.ip_topk(q, p, 100)
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    np.testing.assert_array_equal(s.cpu().numpy(), es)


def _opcheck(op, args, **kw):
    import torch
    torch.library.opcheck(op, args, kw or None, test_utils=("test_schema", "test_faketensor",
                                                            "test_autograd_registration", "test_aot_dispatch_dynamic"))


def test_opcheck_search_ops(dev, drt):
    import torch
    rng = np.random.default_rng(8)
    q = to_dev_bf16(int_bf16(rng, (6, 128), -3, 3), dev)
    p = to_dev_bf16(int_bf16(rng, (5000, 128), -3, 3), dev)
    _opcheck(drt.ip_topk.default, (q, p, 50, 3))
    s, i, _ = drt.ip_topk(q, p, 50, 0)
    _opcheck(drt.topk_merge.default, (torch.stack([s, s]), torch.stack([i, i + 5000]), 60))
    # a valid two-shard protocol run: rows [0, 5000) and [5000, 10000) of a 10000-row corpus
    p2 = to_dev_bf16(int_bf16(rng, (5000, 128), -3, 3), dev)
    _opcheck(drt.dist_sample.default, (q, p, 10000, 50))
    lists = torch.stack([drt.dist_sample(q, p, 10000, 50), drt.dist_sample(q, p2, 10000, 50)])
    _opcheck(drt.dist_tau.default, (lists, 50))
    tau = drt.dist_tau(lists, 50)
    _opcheck(drt.dist_filter.default, (q, p2, 10000, 50, 5000, tau))
    parts = torch.stack([drt.dist_filter(q, p, 10000, 50, 0, tau), drt.dist_filter(q, p2, 10000, 50, 5000, tau)])
    _opcheck(drt.merge_packed.default, (parts, 50, 10000))
    ms, mi, st = drt.merge_packed(parts, 50, 10000)
    assert (st == 0).all()
    es, ei = drt.ip_topk(q, torch.cat([p, p2]), 50, 0)[:2]
    assert torch.equal(mi, ei) and torch.equal(ms, es)


def test_opcheck_score_ce_with_autograd(dev, drt):
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    q = torch.randn(8, 64, device=dev, generator=g, requires_grad=True)
    p = torch.randn(16, 64, device=dev, generator=g, requires_grad=True)
    _opcheck(drt.score_ce_fwd.default, (q, p, 2, 1.0))
    # autograd formula vs torch fp32
    loss, S, _ = drt.score_ce_fwd(q, p, 2, 1.0)
    loss.backward()
    q2, p2 = q.detach().clone().requires_grad_(True), p.detach().clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(q2 @ p2.T, torch.arange(8, device=dev) * 2)
    ref.backward()
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(q.grad, q2.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(p.grad, p2.grad, rtol=1e-4, atol=1e-6)


def test_opcheck_encoder_ops(dev, drt):
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    B, L, H = 2, 32, 256
    ids = torch.randint(1000, 5000, (B, L), device=dev, generator=g)
    mask = torch.ones((B, L), dtype=torch.int64, device=dev)
    mask[1, 20:] = 0
    word = torch.randn(5000, H, device=dev, generator=g) * 0.02
    pos = torch.randn(512, H, device=dev, generator=g) * 0.02
    typ = torch.randn(2, H, device=dev, generator=g) * 0.02
    gam = torch.ones(H, device=dev)
    bet = torch.zeros(H, device=dev)
    _opcheck(drt.embed_ln.default, (ids, None, word, pos, typ, gam, bet, 1e-12))
    h = drt.embed_ln(ids, None, word, pos, typ, gam, bet, 1e-12)
    x = h.view(B * L, H)
    w = (torch.randn(3 * H, H, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(3 * H, device=dev, generator=g) * 0.1
    _opcheck(drt.linear.default, (x, w, b, None, False, False))
    qkv = drt.linear(x, w, b, None, False, False)
    torch.testing.assert_close(qkv.float(), (x.float() @ w.float().T + b), rtol=2e-2, atol=2e-2)
    _opcheck(drt.attention.default, (qkv, mask, B, H // 64, 0.125))
    wo = (torch.randn(H, H, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    _opcheck(drt.linear.default, (x, wo, None, x, False, True))
    y = drt.linear(x, wo, None, x, False, True)
    _opcheck(drt.layernorm.default, (y, gam, bet, 1e-12))
    _opcheck(drt.pool.default, (h, mask, 1))
    _opcheck(drt.l2_normalize.default, (drt.pool(h, mask, 0),))
