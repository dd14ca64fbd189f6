"""GPU: encoder backward building blocks against torch fp32 autograd of the
same forward ops (HF BertModel's LayerNorm / GELU / Linear bias / attention softmax,
transformers modeling_bert.py:164-204, 282-352) on the same bf16 inputs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,H,resid", [(1000, 768, True), (37, 256, False), (4096, 1024, True), (3, 512, False)])
def test_layernorm_bwd_vs_torch(dev, M, H, resid):
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    g = torch.Generator(device=dev).manual_seed(M + H)
    x = (2.0 * torch.randn(M, H, generator=g, device=dev) + 0.3).to(torch.bfloat16)
    gamma = 1.0 + 0.2 * torch.randn(H, generator=g, device=dev)
    beta = 0.1 * torch.randn(H, generator=g, device=dev)
    dy = torch.randn(M, H, generator=g, device=dev).to(torch.bfloat16)
    dres = torch.randn(M, H, generator=g, device=dev).to(torch.bfloat16) if resid else None
    xf = x.float().requires_grad_(True)
    gf = gamma.clone().requires_grad_(True)
    bf = beta.clone().requires_grad_(True)
    torch.nn.functional.layer_norm(xf, (H,), gf, bf, 1e-12).backward(dy.float())
    ref_dx = xf.grad + (dres.float() if resid else 0.0)
    nb = int(lib.drt_layernorm_bwd_workspace(M, H))
    ws = torch.empty((nb + 3) // 4, dtype=torch.float32, device=dev)
    dx = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
    dgam = torch.empty(H, device=dev)
    dbet = torch.empty(H, device=dev)
    _native.check(lib.drt_layernorm_bwd_bf16(dy.data_ptr(), x.data_ptr(), gamma.data_ptr(), 1e-12, M, H,
                                             dres.data_ptr() if resid else None, dx.data_ptr(), dgam.data_ptr(),
                                             dbet.data_ptr(), ws.data_ptr(), nb, _native.stream_ptr(dev)), "ln bwd")
    torch.testing.assert_close(dx.float(), ref_dx, atol=3e-2, rtol=1e-2)
    torch.testing.assert_close(dgam, gf.grad, atol=1e-3 * max(1.0, M ** 0.5), rtol=1e-4)
    torch.testing.assert_close(dbet, bf.grad, atol=1e-3 * max(1.0, M ** 0.5), rtol=1e-4)
    # deterministic: a second run gives identical bits
    dgam2 = torch.empty(H, device=dev)
    _native.check(lib.drt_layernorm_bwd_bf16(dy.data_ptr(), x.data_ptr(), gamma.data_ptr(), 1e-12, M, H,
                                             dres.data_ptr() if resid else None, dx.data_ptr(), dgam2.data_ptr(),
                                             dbet.data_ptr(), ws.data_ptr(), nb, _native.stream_ptr(dev)), "ln bwd")
    assert torch.equal(dgam, dgam2)


@pytest.mark.parametrize("M,N", [(65536, 768), (300, 3072), (1, 64), (255, 100), (5000, 2304)])
def test_colsum_bias_grad_vs_torch(dev, M, N):
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    x = torch.randn(M, N, generator=torch.Generator(device=dev).manual_seed(M), device=dev).to(torch.bfloat16)
    nb = int(lib.drt_colsum_workspace(M, N))
    ws = torch.empty(max(1, (nb + 3) // 4), dtype=torch.float32, device=dev)
    out = torch.empty(N, device=dev)
    _native.check(lib.drt_colsum_bf16(x.data_ptr(), M, N, out.data_ptr(), ws.data_ptr(), nb,
                                      _native.stream_ptr(dev)), "colsum")
    torch.testing.assert_close(out, x.float().sum(0), atol=1e-3 * M ** 0.5, rtol=1e-5)


@pytest.mark.parametrize("n", [65536 * 3072 // 64, 1001, 7])
def test_gelu_bwd_vs_torch(dev, n):
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    g = torch.Generator(device=dev).manual_seed(n)
    pre = (3.0 * torch.randn(n, generator=g, device=dev)).to(torch.bfloat16)
    dy = torch.randn(n, generator=g, device=dev).to(torch.bfloat16)
    xf = pre.float().requires_grad_(True)
    torch.nn.functional.gelu(xf).backward(dy.float())
    dx = torch.empty(n, dtype=torch.bfloat16, device=dev)
    _native.check(lib.drt_gelu_bwd_bf16(dy.data_ptr(), pre.data_ptr(), n, dx.data_ptr(), _native.stream_ptr(dev)),
                  "gelu bwd")
    torch.testing.assert_close(dx.float(), xf.grad, atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("R,C", [(65536, 768), (100, 3072), (1, 1), (129, 65)])
def test_transpose_bf16(dev, R, C):
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    x = torch.randn(R, C, device=dev).to(torch.bfloat16)
    y = torch.empty(C, R, dtype=torch.bfloat16, device=dev)
    _native.check(lib.drt_transpose_bf16(x.data_ptr(), R, C, y.data_ptr(), _native.stream_ptr(dev)), "transpose")
    assert torch.equal(y, x.t().contiguous())


@pytest.mark.parametrize("B,L", [(4, 128), (3, 50), (2, 512), (5, 32)])
def test_attention_lse_vs_torch(dev, B, L):
    """drt_attention_fwd_lse_bf16: ctx unchanged vs drt_attention_bf16, and the per-query
    log-sum-exp of the scaled, key-masked scores against torch fp32 on the same bf16 q/k."""
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    heads, dh = 12, 64
    H = heads * dh
    g = torch.Generator(device=dev).manual_seed(B * L)
    qkv = torch.randn(B * L, 3 * H, generator=g, device=dev).to(torch.bfloat16)
    lens = torch.randint(1, L + 1, (B,), generator=g, device=dev)
    mask = (torch.arange(L, device=dev)[None, :] < lens[:, None]).to(torch.int64)
    ctx0 = torch.empty(B * L, H, dtype=torch.bfloat16, device=dev)
    ctx1 = torch.empty_like(ctx0)
    lse = torch.empty(B, heads, L, device=dev)
    s = _native.stream_ptr(dev)
    scale = 1.0 / dh ** 0.5
    _native.check(lib.drt_attention_bf16(qkv.data_ptr(), mask.data_ptr(), ctx0.data_ptr(), B, L, heads, dh, scale, s), "a")
    _native.check(lib.drt_attention_fwd_lse_bf16(qkv.data_ptr(), mask.data_ptr(), ctx1.data_ptr(), lse.data_ptr(), B, L,
                                                 heads, dh, scale, s), "lse")
    assert torch.equal(ctx0, ctx1)
    q = qkv[:, :H].float().view(B, L, heads, dh).transpose(1, 2)
    k = qkv[:, H:2 * H].float().view(B, L, heads, dh).transpose(1, 2)
    qs = (q * scale).to(torch.bfloat16).float()          # the kernel scales Q in bf16 (exact for dh = 64)
    sc = qs @ k.transpose(-1, -2)
    sc = sc + ((1 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min)
    ref = torch.logsumexp(sc, -1)
    torch.testing.assert_close(lse, ref, atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize("T,N,K", [(16384, 768, 768), (4096, 3072, 768), (1000, 768, 3072), (130, 2304, 768)])
def test_linear_backward_vs_torch(dev, T, N, K):
    """nn.Linear backward on the HIP kernels (dgrad NT GEMM vs the transposed weight, wgrad =
    transposes + split-K NT GEMM with fp32 output, bias = column sums) vs torch fp32 autograd."""
    import torch
    from denseretrievaltoolkits_amd.model.encoder_bwd import linear_backward
    g = torch.Generator(device=dev).manual_seed(T + N + K)
    x = torch.randn(T, K, generator=g, device=dev).to(torch.bfloat16)
    w = (0.05 * torch.randn(N, K, generator=g, device=dev)).to(torch.bfloat16)
    b = torch.randn(N, generator=g, device=dev)
    dy = torch.randn(T, N, generator=g, device=dev).to(torch.bfloat16)
    xf = x.float().requires_grad_(True)
    wf = w.float().requires_grad_(True)
    bf = b.clone().requires_grad_(True)
    torch.nn.functional.linear(xf, wf, bf).backward(dy.float())
    dx, dW, db = linear_backward(dy, x, w.t().contiguous())
    torch.testing.assert_close(dx.float(), xf.grad, atol=3e-2, rtol=1e-2)
    tol = 2e-3 * T ** 0.5
    torch.testing.assert_close(dW, wf.grad, atol=tol, rtol=1e-3)
    torch.testing.assert_close(db, bf.grad, atol=tol, rtol=1e-4)


@pytest.mark.parametrize("B,L", [(4, 128), (3, 50), (6, 32), (2, 100), (3, 156), (2, 160), (2, 129),
                                 (3, 161), (2, 256), (3, 300), (2, 512)])
def test_attention_bwd_vs_torch(dev, B, L):
    """drt_attention_bwd_bf16 (dQ | dK | dV) against torch fp32 autograd of the same attention
    (scaled scores + HF key mask, softmax, P V) on the same bf16 qkv, with padded sequences;
    L > 160 runs the streamed dK/dV + dQ kernels (128-row groups, ragged last group at 161, 300)."""
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    heads, dh = 12, 64
    H = heads * dh
    g = torch.Generator(device=dev).manual_seed(B * 1000 + L)
    qkv = torch.randn(B * L, 3 * H, generator=g, device=dev).to(torch.bfloat16)
    lens = torch.randint(1, L + 1, (B,), generator=g, device=dev)
    lens[0] = L
    mask = (torch.arange(L, device=dev)[None, :] < lens[:, None]).to(torch.int64)
    dctx = torch.randn(B * L, H, generator=g, device=dev).to(torch.bfloat16)
    s = _native.stream_ptr(dev)
    scale = 1.0 / dh ** 0.5
    ctx = torch.empty(B * L, H, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B, heads, L, device=dev)
    _native.check(lib.drt_attention_fwd_lse_bf16(qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), lse.data_ptr(), B, L,
                                                 heads, dh, scale, s), "fwd")
    dqkv = torch.zeros(B * L, 3 * H, dtype=torch.bfloat16, device=dev)
    _native.check(lib.drt_attention_bwd_bf16(qkv.data_ptr(), ctx.data_ptr(), dctx.data_ptr(), lse.data_ptr(),
                                             mask.data_ptr(), dqkv.data_ptr(), B, L, heads, dh, scale, s), "bwd")
    x = qkv.float().requires_grad_(True)
    q = x[:, :H].view(B, L, heads, dh).transpose(1, 2)
    k = x[:, H:2 * H].view(B, L, heads, dh).transpose(1, 2)
    v = x[:, 2 * H:].view(B, L, heads, dh).transpose(1, 2)
    sc = (q * scale) @ k.transpose(-1, -2) + (1 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
    o = torch.softmax(sc, -1) @ v
    o.transpose(1, 2).reshape(B * L, H).backward(dctx.float())
    ref = x.grad
    for name, sl in (("dQ", slice(0, H)), ("dK", slice(H, 2 * H)), ("dV", slice(2 * H, 3 * H))):
        got, want = dqkv[:, sl].float(), ref[:, sl]
        err = (got - want).abs().max().item()
        assert err <= 2e-2 * max(1.0, want.abs().max().item()), (name, err, want.abs().max().item())
        cos = torch.nn.functional.cosine_similarity(got.flatten(), want.flatten(), dim=0).item()
        assert cos > 0.999, (name, cos)
    # drt_attention_train_bwd_bias_bf16: the same dQKV bit for bit plus its column sums (the q / k / v
    # bias gradients) = fp64 sums of the stored bf16 dQKV, to fp32 summation
    dqkv2 = torch.zeros_like(dqkv)
    dbias = torch.empty(3 * H, device=dev)
    nb = int(lib.drt_attention_train_bwd_bias_workspace(B, heads, dh))
    ws = torch.empty((nb + 3) // 4, device=dev)
    _native.check(lib.drt_attention_train_bwd_bias_bf16(qkv.data_ptr(), ctx.data_ptr(), dctx.data_ptr(),
                                                        lse.data_ptr(), mask.data_ptr(), None, dqkv2.data_ptr(), B,
                                                        L, heads, dh, scale, 0.0, 0, 0, dbias.data_ptr(),
                                                        ws.data_ptr(), nb, s), "bwd+bias")
    torch.cuda.synchronize()
    assert torch.equal(dqkv2, dqkv)
    ref_b = dqkv.double().sum(0)
    assert bool(((dbias.double() - ref_b).abs() <= 1e-5 * dqkv.double().abs().sum(0) + 1e-6).all())


@pytest.mark.parametrize("R,C,pad", [(1000, 768, 24), (65536, 3072, 0), (77, 130, 3)])
def test_transpose_bf16_ld(dev, R, C, pad):
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    x = torch.randn(R, C, device=dev).to(torch.bfloat16)
    y = torch.full((C, R + pad), 7.0, dtype=torch.bfloat16, device=dev)
    _native.check(lib.drt_transpose_bf16_ld(x.data_ptr(), R, C, y.data_ptr(), R + pad, _native.stream_ptr(dev)), "t")
    assert torch.equal(y[:, :R], x.t())
    assert bool((y[:, R:] == 7.0).all())


@pytest.mark.parametrize("M,N,K", [(2304, 768, 65536), (768, 3072, 16384), (3072, 768, 131072)])
def test_long_k_split_gemm_vs_torch(dev, M, N, K):
    """Weight-gradient shapes (K = tokens): the 256^2 kernel split over K + fixed-order reduction."""
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    nb = int(lib.drt_linear_workspace(M, N, K))
    assert nb > 0
    g = torch.Generator(device=dev).manual_seed(M + K)
    a = (0.1 * torch.randn(M, K, generator=g, device=dev)).to(torch.bfloat16)
    b = (0.1 * torch.randn(N, K, generator=g, device=dev)).to(torch.bfloat16)
    ws = torch.empty((nb + 3) // 4, device=dev)
    out = torch.empty(M, N, device=dev)
    _native.check(lib.drt_linear_bf16_ws(a.data_ptr(), b.data_ptr(), None, None, out.data_ptr(), M, N, K, 2,
                                         ws.data_ptr(), nb, _native.stream_ptr(dev)), "split gemm")
    ref = a.float() @ b.float().T
    torch.testing.assert_close(out, ref, atol=2e-3 * (K / 4096) ** 0.5, rtol=1e-3)


@pytest.mark.parametrize("T,N,K", [(16384, 768, 768), (131072, 768, 3072), (19968, 2304, 768), (4096, 3072, 768),
                                   (64, 264, 200)])
def test_wgrad_tn_vs_torch_and_transposed_path(dev, T, N, K):
    """dW = dY^T X straight from the token-major operands (drt_linear_wgrad_bf16: the 256^2 GEMM
    in TN mode, ds_read_b64_tr_b16 fragments) vs torch fp32, and bit-identical to the transposed
    path (transposes + NT GEMM) wherever both split the tokens the same way (T % 64 == 0, split)."""
    import torch
    from denseretrievaltoolkits_amd import _native
    from denseretrievaltoolkits_amd.model import encoder_bwd as eb
    g = torch.Generator(device=dev).manual_seed(T + N + K)
    x = torch.randn(T, K, generator=g, device=dev).to(torch.bfloat16)
    dy = torch.randn(T, N, generator=g, device=dev).to(torch.bfloat16)
    eb.WGRAD_TN = True
    try:
        dw_tn = eb.wgrad(dy, x)
        eb.WGRAD_TN = False
        dw_nt = eb.wgrad(dy, x)
    finally:
        eb.WGRAD_TN = True
    ref = dy.float().T @ x.float()
    tol = 2e-3 * T ** 0.5
    torch.testing.assert_close(dw_tn, ref, atol=tol, rtol=1e-3)
    split = _native.load().drt_linear_wgrad_workspace(T, N, K) > 0
    if split and T % 64 == 0:
        assert torch.equal(dw_tn, dw_nt)


def _lin_ex(lib, dev, x, w, bias=None, resid=None, gelu_pre=None, pre_out=None, gelu=False, drop=None, out=None):
    import torch
    from denseretrievaltoolkits_amd import _native
    M, K = x.shape
    N = w.shape[0]
    y = out if out is not None else torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    nb = int(lib.drt_linear_workspace(M, N, K))
    ws = torch.empty(max(1, (nb + 3) // 4), dtype=torch.float32, device=dev)
    p, seed, site = drop if drop is not None else (0.0, 0, 0)
    ptr = (lambda t: t.data_ptr() if t is not None else None)
    _native.check(lib.drt_linear_bf16_ex(x.data_ptr(), w.data_ptr(), ptr(bias), ptr(resid), ptr(gelu_pre),
                                         y.data_ptr(), ptr(pre_out), M, N, K,
                                         (1 if gelu else 0) | (4 if drop is not None else 0), float(p), seed, site,
                                         ws.data_ptr(), nb, _native.stream_ptr(dev)), "drt_linear_bf16_ex")
    return y


@pytest.mark.parametrize("M,N,K", [(65536, 3072, 768), (2000, 3072, 768), (64, 256, 128)])
def test_linear_ex_gelu_pre_outputs_equal_separate_linears(dev, M, N, K):
    """EPI_PRE: one GEMM stores the pre-activation and GELU of it, bit-identical to the linear
    without / with the GELU epilogue (the training forward keeps both)."""
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    g = torch.Generator(device=dev).manual_seed(M + N)
    x = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
    w = (0.05 * torch.randn(N, K, generator=g, device=dev)).to(torch.bfloat16)
    b = 0.1 * torch.randn(N, generator=g, device=dev)
    pre = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    f = _lin_ex(lib, dev, x, w, bias=b, gelu=True, pre_out=pre)
    plain = torch.empty_like(pre)
    act = torch.empty_like(pre)
    for out, flags in ((plain, 0), (act, 1)):
        _native.check(lib.drt_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(), None, out.data_ptr(), M, N, K,
                                          flags, _native.stream_ptr(dev)), "linear")
    torch.cuda.synchronize()
    assert torch.equal(pre, plain)
    assert torch.equal(f, act)


@pytest.mark.parametrize("M,N,K", [(131072, 3072, 768), (4096, 3072, 768), (100, 256, 64)])
def test_linear_ex_dgelu_vs_fp32(dev, M, N, K):
    """EPI_DGELU: dgrad through GELU in the epilogue, vs fp32 torch of (dy W) * GELU'(pre); not
    worse than the unfused dgrad -> drt_gelu_bwd_bf16 path it replaces."""
    import torch
    from denseretrievaltoolkits_amd import _native
    from denseretrievaltoolkits_amd.model.encoder_bwd import gelu_backward
    lib = _native.load()
    g = torch.Generator(device=dev).manual_seed(M + K)
    dy = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
    wt = (0.05 * torch.randn(N, K, generator=g, device=dev)).to(torch.bfloat16)   # W^T rows: [N out, K in]
    pre = (1.5 * torch.randn(M, N, generator=g, device=dev)).to(torch.bfloat16)
    fused = _lin_ex(lib, dev, dy, wt, gelu_pre=pre)
    df = _lin_ex(lib, dev, dy, wt, bias=None)   # plain dgrad (no flags)
    unfused = gelu_backward(df, pre)
    xf = pre.float().requires_grad_(True)
    gl = torch.nn.functional.gelu(xf)
    ref = torch.autograd.grad(gl, xf, (dy.float() @ wt.float().t()))[0]
    err_f = (fused.float() - ref).abs().max().item()
    err_u = (unfused.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err_f <= 1.05 * err_u + 1e-3 * scale, (err_f, err_u, scale)
    assert err_f <= 1e-2 * scale
    # drt_linear_dgelu_bias_bf16: the same dX bit for bit, plus its column sums (the FFN1 bias
    # gradient) -- from the epilogue on the whole-line plan (M 131072, 4096), after the GEMM
    # otherwise -- = fp64 column sums of the stored dX to fp32 summation
    dx2 = torch.empty_like(fused)
    dbias = torch.empty(N, device=dev)
    nb = int(lib.drt_linear_dgelu_bias_workspace(M, N, K))
    ws = torch.empty(max(1, (nb + 3) // 4), dtype=torch.float32, device=dev)
    _native.check(lib.drt_linear_dgelu_bias_bf16(dy.data_ptr(), wt.data_ptr(), pre.data_ptr(), dx2.data_ptr(), M, N, K,
                                                 dbias.data_ptr(), ws.data_ptr(), nb, _native.stream_ptr(dev)),
                  "drt_linear_dgelu_bias_bf16")
    torch.cuda.synchronize()
    assert torch.equal(dx2, fused)
    ref_b = fused.double().sum(0)
    assert bool(((dbias.double() - ref_b).abs() <= 1e-5 * fused.double().abs().sum(0) + 1e-6).all())


@pytest.mark.parametrize("M,N,K,p", [(131072, 768, 3072, 0.1), (16384, 768, 768, 0.1), (300, 768, 64, 0.5)])
def test_linear_ex_dropout_vs_dropout_add(dev, M, N, K, p):
    """EPI_DROP: dropout(x W^T + b) + resid in the epilogue, with drt_dropout_add_bf16's mask:
    same dropped positions, values within the one extra bf16 rounding of the unfused path."""
    import torch
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    g = torch.Generator(device=dev).manual_seed(M + K)
    x = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
    w = (0.05 * torch.randn(N, K, generator=g, device=dev)).to(torch.bfloat16)
    b = 0.1 * torch.randn(N, generator=g, device=dev)
    resid = torch.randn(M, N, generator=g, device=dev).to(torch.bfloat16)
    seed, site = 123456789, 7
    fused = _lin_ex(lib, dev, x, w, bias=b, resid=resid, drop=(p, seed, site))
    y = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    _native.check(lib.drt_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(), None, y.data_ptr(), M, N, K, 0,
                                      _native.stream_ptr(dev)), "linear")
    ref = torch.empty_like(y)
    _native.check(lib.drt_dropout_add_bf16(y.data_ptr(), resid.data_ptr(), y.numel(), p, seed, site,
                                           ref.data_ptr(), _native.stream_ptr(dev)), "dropout_add")
    torch.cuda.synchronize()
    dropped_ref = ref == resid
    keep_frac = 1.0 - (fused == resid).float().mean().item()
    assert abs(keep_frac - (1.0 - p)) < 0.02
    # wherever the unfused path kept the element, both agree to one bf16 rounding of the sum
    torch.testing.assert_close(fused.float(), ref.float(), atol=2e-2, rtol=1e-2)
    assert ((fused == resid) | ~dropped_ref).float().mean().item() > 0.999


@pytest.mark.parametrize("M,H", [(131072, 768), (37, 256)])
def test_layernorm_bwd_drop_output_equals_dropout_kernel(dev, M, H):
    """drt_layernorm_bwd_drop_bf16: dx identical to drt_layernorm_bwd_bf16 and dx_drop bit-identical
    to drt_dropout_add_bf16(dx) with the same (p, seed, site)."""
    import torch
    from denseretrievaltoolkits_amd import _native
    from denseretrievaltoolkits_amd.model.encoder_bwd import layernorm_backward
    lib = _native.load()
    g = torch.Generator(device=dev).manual_seed(M + H)
    x = (2.0 * torch.randn(M, H, generator=g, device=dev)).to(torch.bfloat16)
    gamma = 1.0 + 0.2 * torch.randn(H, generator=g, device=dev)
    dy = torch.randn(M, H, generator=g, device=dev).to(torch.bfloat16)
    dx, dg, db, dxd = layernorm_backward(dy, x, gamma, 1e-12, drop=(0.1, 99, 5))
    dx0, dg0, db0 = layernorm_backward(dy, x, gamma, 1e-12)
    ref = torch.empty_like(dx)
    _native.check(lib.drt_dropout_add_bf16(dx0.data_ptr(), None, dx0.numel(), 0.1, 99, 5, ref.data_ptr(),
                                           _native.stream_ptr(dev)), "dropout")
    torch.cuda.synchronize()
    assert torch.equal(dx, dx0) and torch.equal(dg, dg0) and torch.equal(db, db0)
    assert torch.equal(dxd, ref)
    # drt_layernorm_bwd_sum_bf16: the same outputs plus the column sums of what it hands down
    # (the linear-bias gradient) = fp64 column sums of the stored bf16 gradient, to fp32 summation
    dx_s, dg_s, db_s, dxd_s, sd = layernorm_backward(dy, x, gamma, 1e-12, drop=(0.1, 99, 5), want_sum=True)
    dx_n, _, _, sn = layernorm_backward(dy, x, gamma, 1e-12, want_sum=True)
    assert torch.equal(dx_s, dx) and torch.equal(dxd_s, dxd) and torch.equal(dg_s, dg) and torch.equal(db_s, db)
    for s_, t_ in ((sd, dxd), (sn, dx_n)):
        ref_s = t_.double().sum(0)
        tol = 1e-5 * t_.double().abs().sum(0) + 1e-6
        assert bool(((s_.double() - ref_s).abs() <= tol).all())


@pytest.mark.parametrize("L,B", [(128, 6), (156, 5), (37, 9), (32, 4), (200, 3), (512, 2)])
def test_attention_dropout_bits_vs_hash_and_torch(dev, L, B):
    """drt_attention_train_fwd_bits_bf16 writes the attention-dropout keep mask as bits (the forward's
    outputs do not change, the bits are the hash's keep decisions); the backward that reads them and
    the one that draws the same bits again from the hash (C-ABI callers without bits) both
    match torch fp32 autograd of the same dropped attention (the mask from the host restatement of the
    pairwise attention hash).  L > 160 (streamed backward): the bits are required -- a backward
    without them is refused."""
    import torch
    from denseretrievaltoolkits_amd import _native
    from tests.test_train_tower_gpu import _attn_keep_py, _attn_keep_torch
    lib = _native.load()
    s = _native.stream_ptr(dev)
    heads, dh, p, seed, site = 12, 64, 0.1, 77, 3
    H = heads * dh
    scale = 1.0 / dh ** 0.5
    g = torch.Generator(device=dev).manual_seed(L)
    qkv = (0.5 * torch.randn(B * L, 3 * H, generator=g, device=dev)).to(torch.bfloat16)
    dctx = (0.1 * torch.randn(B * L, H, generator=g, device=dev)).to(torch.bfloat16)
    mask = torch.ones(B, L, dtype=torch.int64, device=dev)
    mask[1, L - 5:] = 0
    nkb = (L + 31) // 32
    outs = {}
    for use_bits in (False, True):
        ctx = torch.empty(B * L, H, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(B * heads * L, dtype=torch.float32, device=dev)
        bits = torch.full((B, heads, L, nkb), -1, dtype=torch.int32, device=dev) if use_bits else None
        _native.check(lib.drt_attention_train_fwd_bits_bf16(qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(),
                                                            lse.data_ptr(), bits.data_ptr() if use_bits else None,
                                                            B, L, heads, dh, scale, p, seed, site, s), "fwd")
        dqkv = torch.empty_like(qkv)
        rc = lib.drt_attention_train_bwd_bits_bf16(qkv.data_ptr(), ctx.data_ptr(), dctx.data_ptr(), lse.data_ptr(),
                                                   mask.data_ptr(), bits.data_ptr() if use_bits else None,
                                                   dqkv.data_ptr(), B, L, heads, dh, scale, p, seed, site, s)
        if L > 160 and not use_bits:
            assert rc != 0
            dqkv = None
        else:
            _native.check(rc, "bwd")
        torch.cuda.synchronize()
        outs[use_bits] = (ctx, lse, dqkv, bits)
    assert torch.equal(outs[False][0], outs[True][0]) and torch.equal(outs[False][1], outs[True][1])
    # torch fp32 reference with the same keep mask (host restatement of the attention hash)
    keep = _attn_keep_torch(seed, site, B, heads, L, p, dev).float()
    x = qkv.float().requires_grad_(True)
    q = x[:, :H].view(B, L, heads, dh).transpose(1, 2)
    k = x[:, H:2 * H].view(B, L, heads, dh).transpose(1, 2)
    v = x[:, 2 * H:].view(B, L, heads, dh).transpose(1, 2)
    sc = (q * scale) @ k.transpose(-1, -2) + (1 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
    o = (torch.softmax(sc, -1) * keep / (1 - p)) @ v
    o.transpose(1, 2).reshape(B * L, H).backward(dctx.float())
    ref = x.grad
    for use_bits in (False, True):
        dq = outs[use_bits][2]
        if dq is None:
            continue
        for name, sl in (("dQ", slice(0, H)), ("dK", slice(H, 2 * H)), ("dV", slice(2 * H, 3 * H))):
            got, want = dq[:, sl].float(), ref[:, sl]
            cos = torch.nn.functional.cosine_similarity(got.flatten(), want.flatten(), dim=0).item()
            assert cos > 0.999, (use_bits, name, cos)
            err = (got - want).abs().max().item()
            assert err <= 2e-2 * max(1.0, want.abs().max().item()), (use_bits, name, err)
    # the bits are the hash's keep decisions
    bb, hd = B - 1, heads // 2
    w = outs[True][3][bb, hd].cpu().numpy().astype(np.uint32)
    for qq in (0, L // 2, L - 1):
        for key in range(L):
            want = _attn_keep_py(seed, site, (bb * heads + hd) * L + qq, key, p)
            assert bool((w[qq, key >> 5] >> (key & 31)) & 1) == want, (qq, key)
