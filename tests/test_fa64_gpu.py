"""Head-dim-64 flash attention (csrc/kernels/flash_attn_d64.hip: 8-wave LDS-DMA kernels with
in-kernel dropout and packed-QKV strides) against a plain PyTorch fp32 reference of the same op
(with dropout: the keep mask probed through V = I), and against the generic 4-wave kernels
(PHA_FA64=0) without dropout."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(q, k, v, causal, scale, keep=None, rate=0.0):
    qt, kt, vt = (t.float().transpose(1, 2) for t in (q, k, v))
    if kt.shape[1] != qt.shape[1]:
        g = qt.shape[1] // kt.shape[1]
        kt, vt = kt.repeat_interleave(g, 1), vt.repeat_interleave(g, 1)
    s = (qt @ kt.transpose(-1, -2)) * scale
    if causal:
        S, Sk = s.shape[-2:]
        s = s.masked_fill(torch.ones(S, Sk, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    p = torch.softmax(s, -1)
    if keep is not None:
        p = p * keep / (1.0 - rate)
    return (p @ vt).transpose(1, 2)


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()


@pytest.mark.parametrize("B,S,Sk,H,Hk", [(2, 512, 512, 4, 4), (1, 200, 200, 3, 3), (2, 300, 136, 4, 2),
                                         (1, 64, 64, 2, 2), (1, 1000, 1000, 2, 1)])
@pytest.mark.parametrize("causal", [False, True])
def test_fa64_matches_fp32_reference(B, S, Sk, H, Hk, causal):
    from paddle_hackathon_amd.ops import hip
    if causal and S != Sk:
        pytest.skip("causal attention with S != Sk is bottom-right aligned by no caller")
    g = torch.Generator(device="cuda").manual_seed(S + Sk + H)
    q = torch.randn(B, S, H, 64, device="cuda", generator=g).bfloat16().requires_grad_()
    k = torch.randn(B, Sk, Hk, 64, device="cuda", generator=g).bfloat16().requires_grad_()
    v = torch.randn(B, Sk, Hk, 64, device="cuda", generator=g).bfloat16().requires_grad_()
    sc = 1.0 / math.sqrt(64)
    o = hip.FlashAttentionExt.apply(q, k, v, causal, sc, None, 0.0)
    assert o.grad_fn is not None
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    ref = _ref(qr, kr, vr, causal, sc)
    assert _rel(o, ref) < 2e-2
    do = torch.randn_like(o)
    g1 = torch.autograd.grad(o, (q, k, v), do)
    g2 = torch.autograd.grad(ref, (qr, kr, vr), do.float())
    for a, b in zip(g1, g2):
        assert _rel(a, b) < 3e-2


@pytest.mark.parametrize("rate", [0.1, 0.5])
@pytest.mark.parametrize("causal", [False, True])
def test_fa64_dropout_mask_density_and_grads(rate, causal):
    """the keep mask read back through V = I has density 1 - rate, and forward + backward equal the
    fp32 reference with that same mask (so the backward regenerates the forward's mask)"""
    from paddle_hackathon_amd import ops
    B, S, H = 2, 192, 2
    torch.manual_seed(11)
    q = torch.randn(B, S, H, 64, device="cuda").bfloat16()
    k = torch.randn(B, S, H, 64, device="cuda").bfloat16()
    eye = torch.eye(S, device="cuda").bfloat16()
    # V = I needs D = S: probe the mask 64 keys at a time (the kernel's head dim), same seed
    keep = torch.zeros(B, H, S, S, device="cuda")
    for c in range(0, S, 64):
        vi = eye[:, c:c + 64][None, :, None, :].expand(B, S, H, 64).contiguous()
        torch.manual_seed(123)
        pd = ops.flash_attention(q, k, vi, causal=causal, dropout_p=rate, training=True).float()   # [B, S, H, 64]
        keep[:, :, :, c:c + 64] = (pd != 0).transpose(1, 2).float()
    valid = torch.ones(S, S, device="cuda") if not causal else torch.ones(S, S, device="cuda").tril()
    frac = (keep * valid).sum() / (valid.sum() * B * H)
    assert abs(frac.item() - (1 - rate)) < 0.03, frac
    v = torch.randn(B, S, H, 64, device="cuda").bfloat16()
    qg, kg, vg = (t.clone().requires_grad_() for t in (q, k, v))
    torch.manual_seed(123)
    o = ops.flash_attention(qg, kg, vg, causal=causal, dropout_p=rate, training=True)
    sc = 1.0 / 8.0
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    ref = _ref(qr, kr, vr, causal, sc, keep, rate)
    assert _rel(o, ref) < 3e-2
    do = torch.randn_like(o)
    g1 = torch.autograd.grad(o, (qg, kg, vg), do)
    g2 = torch.autograd.grad(ref, (qr, kr, vr), do.float())
    for a, b in zip(g1, g2):
        assert _rel(a, b) < 3e-2


@pytest.mark.parametrize("rate", [0.0])
def test_fa64_packed_matches_generic_kernels(rate, monkeypatch):
    """BERT's packed [B, S, H, 3 * 64] entry on the new kernels (read in place, gradients written
    through the packed strides) vs the generic 4-wave kernels (their dropout draws differ: the D = 64
    kernels' fa64_draw; dropout is checked against the probed mask in the test above)"""
    from paddle_hackathon_amd.ops import hip
    B, S, H = 2, 512, 4
    torch.manual_seed(3)
    qkv = torch.randn(B, S, H, 192, device="cuda").bfloat16()
    do = torch.randn(B, S, H, 64, device="cuda").bfloat16()
    outs = []
    for on in ("1", "0"):
        monkeypatch.setenv("PHA_FA64", on)
        a = qkv.clone().requires_grad_()
        torch.manual_seed(99)
        o = hip.flash_attention_packed_ext(a, False, None, None, rate)
        (gq,) = torch.autograd.grad(o, a, do)
        outs.append((o.float(), gq.float()))
    (o1, g1), (o0, g0) = outs
    assert _rel(o1, o0) < 2e-2
    assert _rel(g1, g0) < 3e-2


def test_fa64_kernels_are_the_ones_running(monkeypatch):
    """with PHA_FA64 on (the default) the D = 64 ext path must not reach the generic ext entry"""
    from paddle_hackathon_amd.ops import hip
    L = hip._L()
    called = {"ext": 0}
    orig = hip.FlashAttentionExt.forward

    def spy(ctx, *a):
        r = orig(ctx, *a)
        called["ext"] += 0 if getattr(ctx, "fa64", False) else 1
        return r
    monkeypatch.setattr(hip.FlashAttentionExt, "forward", staticmethod(spy))
    q = torch.randn(1, 128, 2, 64, device="cuda").bfloat16()
    hip.FlashAttentionExt.apply(q, q, q, False, 0.125, None, 0.1)
    assert called["ext"] == 0 and hasattr(L, "pha_fa64_fwd")


@pytest.mark.parametrize("causal", [False, True])
def test_fa64_plain_entry_matches_generic(causal, monkeypatch):
    """ops.flash_attention without mask / dropout at D = 64 (FlashAttention: GPT-2-sized models)
    runs the new kernels; same result as the generic 4-wave kernels"""
    from paddle_hackathon_amd import ops
    torch.manual_seed(1)
    q, k, v = (torch.randn(2, 384, 6, 64, device="cuda").bfloat16() for _ in range(3))
    do = torch.randn_like(q)
    res = []
    for on in ("1", "0"):
        monkeypatch.setenv("PHA_FA64", on)
        qg, kg, vg = (t.clone().requires_grad_() for t in (q, k, v))
        o = ops.flash_attention(qg, kg, vg, causal=causal)
        res.append((o.float(),) + tuple(x.float() for x in torch.autograd.grad(o, (qg, kg, vg), do)))
    for a, b in zip(*res):
        assert _rel(a, b) < 2e-2


@pytest.mark.parametrize("causal", [False, True])
def test_fa64_stored_keep_bits_equal_rehashed_mask(causal, monkeypatch):
    """the backward reading the forward's keep bits (default) is bitwise equal to the backward that
    re-hashes the mask (PHA_FA64_MASKBITS=0), incl. a ragged key count"""
    from paddle_hackathon_amd.ops import hip
    torch.manual_seed(4)
    B, S, H = 2, 328, 3
    qkv = torch.randn(B, S, H, 192, device="cuda").bfloat16()
    do = torch.randn(B, S, H, 64, device="cuda").bfloat16()
    res = []
    for mb in ("1", "0"):
        monkeypatch.setenv("PHA_FA64_MASKBITS", mb)
        a = qkv.clone().requires_grad_()
        torch.manual_seed(21)
        o = hip.flash_attention_packed_ext(a, causal, None, None, 0.1)
        (g,) = torch.autograd.grad(o, a, do)
        res.append((o, g))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("kind", ["keypad", "full", "bool"])
@pytest.mark.parametrize("causal", [False, True])
def test_fa64_additive_masks_match_fp32(kind, causal):
    """additive key-padding [B,1,1,Sk], full [B,H,S,Sk] and boolean masks on the D = 64 kernels (the
    bias / scale starts the score accumulators; key-padding columns hoisted in the dK/dV kernel)"""
    from paddle_hackathon_amd import ops
    from paddle_hackathon_amd.ops import hip
    B, S, H = 2, 200, 3
    torch.manual_seed(8)
    q, k, v = (torch.randn(B, S, H, 64, device="cuda").bfloat16().requires_grad_() for _ in range(3))
    if kind == "keypad":
        mask = torch.where(torch.arange(S, device="cuda") < S - 23, 0.0, -1e4).reshape(1, 1, 1, S).expand(B, 1, 1, S)
        bias = mask
    elif kind == "full":
        mask = torch.randn(B, H, S, S, device="cuda")
        bias = mask
    else:
        mask = (torch.rand(B, 1, S, S, device="cuda") > 0.2) | torch.eye(S, device="cuda", dtype=torch.bool)
        bias = torch.zeros(mask.shape, device="cuda").masked_fill(~mask, float("-inf"))
    o = ops.flash_attention(q, k, v, causal=causal, mask=mask)
    assert o.grad_fn is not None and getattr(o.grad_fn, "_raw_saved_self", None) is None
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    qt, kt, vt = (t.transpose(1, 2) for t in (qr, kr, vr))
    s = qt @ kt.transpose(-1, -2) / 8.0 + bias
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device="cuda").triu(1), float("-inf"))
    ref = (torch.softmax(s, -1) @ vt).transpose(1, 2)
    assert _rel(o, ref) < 2e-2
    do = torch.randn_like(o)
    g1 = torch.autograd.grad(o, (q, k, v), do)
    g2 = torch.autograd.grad(ref, (qr, kr, vr), do.float())
    for a, b in zip(g1, g2):
        assert _rel(a, b) < 3e-2
    assert hip._fa64_on(64, mask, S)


@pytest.mark.parametrize("waves", ["4", "8"])
@pytest.mark.parametrize("causal,rate", [(False, 0.1), (True, 0.0), (False, 0.0)])
def test_fa64_dkdv_workgroup_sizes_agree(waves, causal, rate, monkeypatch):
    """the dK/dV kernel at 4 waves (128 keys per workgroup) and 8 waves (256 keys) computes the same
    gradients (same per-key accumulation order: bitwise), ragged key count, stored keep bits"""
    from paddle_hackathon_amd.ops import hip
    torch.manual_seed(6)
    B, S, H = 2, 456, 3
    qkv = torch.randn(B, S, H, 192, device="cuda").bfloat16()
    do = torch.randn(B, S, H, 64, device="cuda").bfloat16()
    res = []
    for w in (waves, "8"):
        monkeypatch.setenv("PHA_FA64_DKDV_WAVES", w)
        a = qkv.clone().requires_grad_()
        torch.manual_seed(31)
        o = hip.flash_attention_packed_ext(a, causal, None, None, rate)
        (g,) = torch.autograd.grad(o, a, do)
        res.append(g)
    assert torch.equal(res[0], res[1])
