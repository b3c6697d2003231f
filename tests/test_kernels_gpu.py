"""Numerics of the gfx950 HIP kernels vs plain PyTorch fp32 references (GPU only).

Each test asserts the native library is the code path that ran (no silent fallback).
"""
import math

import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _native():
    from paddle_hackathon_amd.ops import _lib
    assert _lib.native_available(), "libpha_kernels.so must be loaded on a GPU run"
    yield


def _tol(dt):
    return {torch.float32: 2e-5, torch.bfloat16: 2e-2, torch.float16: 2e-3}[dt]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H", [64, 768, 1000 * 0 + 1024, 2048, 2056, 4096])
def test_layer_norm_fwd_bwd(dt, H):
    from paddle_hackathon_amd.ops import hip
    torch.manual_seed(0)
    rows = 37
    x = torch.randn(rows, H, device="cuda").to(dt)
    w = (torch.rand(H, device="cuda") + 0.5).to(dt)
    b = torch.randn(H, device="cuda").to(dt)
    y, mean, rstd = hip.layer_norm_fwd(x, w, b, 1e-5)
    ref = TF.layer_norm(x.float(), [H], w.float(), b.float(), 1e-5)
    assert torch.allclose(y.float(), ref, atol=_tol(dt) * 4, rtol=_tol(dt))
    dy = torch.randn_like(x)
    dx, dw, db = hip.layer_norm_bwd(dy, x, w, mean, rstd, True)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    br = b.float().requires_grad_(True)
    TF.layer_norm(xr, [H], wr, br, 1e-5).backward(dy.float())
    assert torch.allclose(dx.float(), xr.grad, atol=_tol(dt) * 8, rtol=_tol(dt) * 2)
    assert torch.allclose(dw.float(), wr.grad, atol=_tol(dt) * 40, rtol=_tol(dt) * 2)
    assert torch.allclose(db.float(), br.grad, atol=_tol(dt) * 40, rtol=_tol(dt) * 2)


def test_layer_norm_fp32_weight_bf16_input():
    from paddle_hackathon_amd.ops import hip
    x = torch.randn(64, 2048, device="cuda").bfloat16()
    w = torch.rand(2048, device="cuda") + 0.5
    b = torch.randn(2048, device="cuda")
    y, _, _ = hip.layer_norm_fwd(x, w, b, 1e-5)
    ref = TF.layer_norm(x.float(), [2048], w, b, 1e-5)
    assert torch.allclose(y.float(), ref, atol=5e-2, rtol=2e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H", [128, 1024, 2048, 4096])
def test_softmax(dt, H):
    from paddle_hackathon_amd.ops import hip
    x = (torch.randn(50, H, device="cuda") * 3).to(dt)
    y = hip.softmax_fwd(x)
    ref = torch.softmax(x.float(), -1)
    assert torch.allclose(y.float(), ref, atol=_tol(dt), rtol=_tol(dt) * 2)
    dy = torch.randn_like(x)
    dx = hip.softmax_bwd(dy, y)
    xr = x.float().requires_grad_(True)
    torch.softmax(xr, -1).backward(dy.float())
    assert torch.allclose(dx.float(), xr.grad, atol=_tol(dt) * 2, rtol=_tol(dt) * 4)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("V", [512, 50304, 32000])
def test_softmax_cross_entropy(dt, V):
    from paddle_hackathon_amd import ops
    rows = 67
    logits = (torch.randn(rows, V, device="cuda") * 2).to(dt).requires_grad_(True)
    labels = torch.randint(0, V, (rows,), device="cuda")
    labels[3] = -100
    loss = ops.softmax_cross_entropy(logits, labels, -100)
    ref_l = logits.detach().float().requires_grad_(True)
    ref = TF.cross_entropy(ref_l, labels, reduction="none", ignore_index=-100)
    assert torch.allclose(loss, ref, atol=1e-3 if dt == torch.float32 else 2e-2, rtol=1e-3)
    g = torch.rand(rows, device="cuda")
    loss.backward(g)
    ref.backward(g)
    assert torch.allclose(logits.grad.float(), ref_l.grad, atol=1e-5 if dt == torch.float32 else 2e-3, rtol=2e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("approx", [False, True])
def test_bias_gelu(dt, approx):
    from paddle_hackathon_amd import ops
    x = torch.randn(33, 4096, device="cuda").to(dt).requires_grad_(True)
    b = torch.randn(4096, device="cuda").to(dt).requires_grad_(True)
    y = ops.bias_gelu(x, b, approx)
    xr = x.detach().float().requires_grad_(True)
    br = b.detach().float().requires_grad_(True)
    ref = TF.gelu(xr + br, approximate="tanh" if approx else "none")
    assert torch.allclose(y.float(), ref, atol=_tol(dt) * 2, rtol=_tol(dt))
    g = torch.randn_like(ref)
    y.backward(g.to(dt))
    ref.backward(g)
    assert torch.allclose(x.grad.float(), xr.grad, atol=_tol(dt) * 4, rtol=_tol(dt) * 2)
    assert torch.allclose(b.grad.float(), br.grad, atol=_tol(dt) * 60, rtol=_tol(dt) * 2)


def test_embedding_fwd_bwd():
    from paddle_hackathon_amd import ops
    w = torch.randn(1000, 256, device="cuda").bfloat16().requires_grad_(True)
    ids = torch.randint(0, 1000, (4, 77), device="cuda")
    y = ops.embedding(ids, w)
    assert torch.equal(y, w.detach()[ids])
    y.float().sum().backward()
    ref = torch.zeros(1000, 256, device="cuda").index_add_(0, ids.reshape(-1), torch.ones(ids.numel(), 256, device="cuda"))
    assert torch.allclose(w.grad.float(), ref, atol=1e-2)


@pytest.mark.parametrize("pdt", [torch.float32, torch.bfloat16])
def test_multi_tensor_adamw(pdt):
    from paddle_hackathon_amd.ops import hip, fused
    torch.manual_seed(0)
    shapes = [(1000,), (37, 129), (2048, 64), (3,)]
    ps = [torch.randn(s, device="cuda").to(pdt) for s in shapes]
    gs = [torch.randn(s, device="cuda").to(pdt) for s in shapes]
    ms = [torch.zeros(s, device="cuda") for s in shapes]
    vs = [torch.zeros(s, device="cuda") for s in shapes]
    masters = [p.float().clone() if pdt != torch.float32 else None for p in ps]
    # reference: CPU path of the same op in fp32
    rp = [p.float().cpu().clone() for p in ps]
    rg = [g.float().cpu() for g in gs]
    rm = [torch.zeros(s) for s in shapes]
    rv = [torch.zeros(s) for s in shapes]
    for step in (1, 2, 3):
        hip.multi_tensor_adam(ps, gs, ms, vs, masters, 1e-2, 0.9, 0.95, 1e-8, step, 0.0, True, None, 1.0, [0.1] * 4)
        fused.fused_adam_(rp, rg, rm, rv, None, 1e-2, 0.9, 0.95, 1e-8, step, 0.1, True, None, 1.0)
    for i in range(len(shapes)):
        got = (masters[i] if masters[i] is not None else ps[i]).float().cpu()
        assert torch.allclose(got, rp[i], atol=1e-5, rtol=1e-5), i
        assert torch.allclose(ms[i].cpu(), rm[i], atol=1e-6)


def test_multi_tensor_l2norm():
    from paddle_hackathon_amd.ops import hip
    ts = [torch.randn(s, device="cuda").bfloat16() for s in [(5000,), (128, 300), (7,)]]
    got = hip.multi_tensor_l2norm_sq(ts)
    ref = sum(t.float().pow(2).sum() for t in ts)
    assert torch.allclose(got, ref, rtol=1e-4)


def test_gpt_tiny_train_step_gpu():
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.models import gpt_config, GPTForPretraining
    paddle.set_device("gpu:0")
    paddle.seed(0)
    cfg = gpt_config("gpt-tiny")
    m = paddle.amp.decorate(GPTForPretraining(cfg), level="O2", dtype="bfloat16")
    opt = paddle.optimizer.AdamW(1e-3, parameters=m.parameters())
    ids = paddle.randint(0, cfg.vocab_size, [4, 64])
    losses = []
    for _ in range(30):
        loss = m(ids, ids)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(loss.item())
    assert losses[-1] < losses[0] - 1.0, losses


def _ref_attn(q, k, v, causal, scale=None):
    B, S, H, D = q.shape
    Hk = k.shape[2]
    if Hk != H:
        k = k.repeat_interleave(H // Hk, dim=2)
        v = v.repeat_interleave(H // Hk, dim=2)
    qt, kt, vt = (t.float().transpose(1, 2) for t in (q, k, v))
    o = TF.scaled_dot_product_attention(qt, kt, vt, is_causal=causal, scale=scale)
    return o.transpose(1, 2)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("S", [128, 200, 512])
def test_flash_attention_fwd_bwd(dt, D, causal, S):
    from paddle_hackathon_amd.ops import hip
    torch.manual_seed(0)
    B, H = 2, 3
    q = torch.randn(B, S, H, D, device="cuda").to(dt).requires_grad_(True)
    k = torch.randn(B, S, H, D, device="cuda").to(dt).requires_grad_(True)
    v = torch.randn(B, S, H, D, device="cuda").to(dt).requires_grad_(True)
    assert hip.flash_attn_supported(q, k, v, 0.0)
    o = hip.FlashAttention.apply(q, k, v, causal, None)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = _ref_attn(qr, kr, vr, causal)
    assert (o.float() - ref).abs().max().item() < 2e-2, (o.float() - ref).abs().max().item()
    g = torch.randn_like(ref)
    o.backward(g.to(dt))
    ref.backward(g)
    for got, want, name in ((q.grad, qr.grad, "dq"), (k.grad, kr.grad, "dk"), (v.grad, vr.grad, "dv")):
        err = (got.float() - want).abs().max().item()
        scale = want.abs().max().item()
        assert err < 3e-2 * max(1.0, scale), (name, err, scale)


def test_flash_attention_gqa():
    from paddle_hackathon_amd.ops import hip
    torch.manual_seed(0)
    q = torch.randn(1, 256, 8, 128, device="cuda").bfloat16()
    k = torch.randn(1, 256, 2, 128, device="cuda").bfloat16()
    v = torch.randn(1, 256, 2, 128, device="cuda").bfloat16()
    o = hip.FlashAttention.apply(q, k, v, True, None)
    ref = _ref_attn(q, k, v, True)
    assert (o.float() - ref).abs().max().item() < 2e-2
