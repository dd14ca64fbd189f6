"""CPU: the torch.ops.drt custom-op library loads, every operator has its schema and a fake
(meta) implementation with the right output shapes (FakeTensor tracing needs no GPU), and
real CPU tensors are refused by the dispatcher (no CPU fallback exists)."""
import pytest
import torch

OPS = ["ip_topk", "ip_topk_resolve", "topk_merge", "dist_sample", "dist_tau", "dist_filter", "dist_filter_lists", "dist_filter_lists_into", "dist_filter_into", "merge_packed",
       "score_ce_fwd", "score_ce_bwd", "embed_ln", "linear", "attention", "layernorm", "pool", "l2_normalize"]


@pytest.fixture(scope="module")
def drt():
    from denseretrievaltoolkits_amd import ops
    return ops.load()


def test_every_op_registered(drt):
    for name in OPS:
        op = getattr(torch.ops.drt, name)
        assert op.default._schema.name == f"drt::{name}"
    assert "Tensor(a!) scores" in str(torch.ops.drt.ip_topk.out._schema)


def test_fake_shapes(drt):
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        q = torch.empty(5, 768, dtype=torch.bfloat16, device="cuda")
        p = torch.empty(1000, 768, dtype=torch.bfloat16, device="cuda")
        s, i, st = drt.ip_topk(q, p, 10, 0)
        assert (s.shape, s.dtype, i.dtype, st.shape, st.dtype) == ((5, 10), torch.float32, torch.int64, (5,),
                                                                   torch.int32)
        assert drt.ip_topk.out(q, p, 10, 0, scores=s, ids=i, status=st) is None
        ms, mi = drt.topk_merge(torch.empty(3, 5, 10, device="cuda"), torch.empty(3, 5, 10, dtype=torch.int64,
                                                                                  device="cuda"), 7)
        assert ms.shape == (5, 7) and mi.dtype == torch.int64
        best = drt.dist_sample(q, p, 8000, 1000)
        assert best.shape[0] == 5 and best.dtype == torch.int32
        tau = drt.dist_tau(torch.empty(4, 5, best.shape[1], dtype=torch.int32, device="cuda"), 1000)
        assert tau.shape == (5,)
        pk = drt.dist_filter(q, p, 8000, 1000, 0, tau)
        assert pk.shape == (5, 1001) and pk.dtype == torch.int64
        s2, i2, st2 = drt.merge_packed(torch.empty(4, 5, 1001, dtype=torch.int64, device="cuda"), 1000, 8000)
        assert s2.shape == (5, 1000) and st2.shape == (5,)
        qf = torch.empty(8, 768, device="cuda", requires_grad=True)
        pf = torch.empty(16, 768, device="cuda", requires_grad=True)
        loss, S, lse = drt.score_ce_fwd(qf, pf, 2, 1.0)
        assert loss.shape == () and S.shape == (8, 16) and lse.shape == (8,)
        ids = torch.empty(2, 32, dtype=torch.int64, device="cuda")
        h = drt.embed_ln(ids, None, torch.empty(30522, 768, device="cuda"), torch.empty(512, 768, device="cuda"),
                         torch.empty(2, 768, device="cuda"), torch.empty(768, device="cuda"),
                         torch.empty(768, device="cuda"), 1e-12)
        assert h.shape == (2, 32, 768) and h.dtype == torch.bfloat16
        x = h.view(64, 768)
        y = drt.linear(x, torch.empty(2304, 768, dtype=torch.bfloat16, device="cuda"), None, None, False, True)
        assert y.shape == (64, 2304) and y.dtype == torch.float32
        ctx = drt.attention(torch.empty(64, 2304, dtype=torch.bfloat16, device="cuda"), None, 2, 12, 0.125)
        assert ctx.shape == (64, 768)
        assert drt.layernorm(y[:, :768], torch.empty(768, device="cuda"), torch.empty(768, device="cuda"),
                             1e-12).dtype == torch.bfloat16
        assert drt.pool(h, None, 1).shape == (2, 768)
        assert drt.l2_normalize(torch.empty(2, 768, device="cuda")).shape == (2, 768)


def test_cpu_tensors_refused(drt):
    with pytest.raises(NotImplementedError):
        drt.ip_topk(torch.zeros(2, 64, dtype=torch.bfloat16), torch.zeros(5, 64, dtype=torch.bfloat16), 3, 0)
    from denseretrievaltoolkits_amd import kernels
    with pytest.raises(ValueError, match="GPU only"):
        kernels.ip_topk(torch.zeros(2, 64, dtype=torch.bfloat16), torch.zeros(5, 64, dtype=torch.bfloat16), 3)
