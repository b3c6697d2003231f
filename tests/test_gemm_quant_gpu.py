"""GPU numerics of the round-4 kernels against fp32 torch references:
  * paddle.matmul / mm / bmm / bias-less linear through ops/gemm.py matmul (NN / NT / TN layouts
    with autograd), no fallback and, under PHA_GEMM_IMPL=own, no library product;
  * the 8-wave NT GEMM (csrc/kernels/gemm8w.hip);
  * the fake-quantization kernels (csrc/kernels/quant.hip) — reference fake_quantize_op.cu.h."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _r(*s, dtype=torch.bfloat16, g=None):
    return (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(dtype)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False)])
@pytest.mark.parametrize("M,N,K", [(256, 512, 128), (100, 72, 40), (2, 3, 5)])
def test_paddle_matmul_own_layouts(ta, tb, M, N, K, monkeypatch):
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    monkeypatch.setenv("PHA_GEMM_IMPL", "own")
    paddle.set_device("gpu")
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = _r(*((K, M) if ta else (M, K)), g=g)
    b = _r(*((N, K) if tb else (K, N)), g=g)
    x, y = paddle.to_tensor(a), paddle.to_tensor(b)
    x.stop_gradient = y.stop_gradient = False
    fallback.reset()
    out = paddle.matmul(x, y, transpose_x=ta, transpose_y=tb)
    gout = _r(M, N, g=g)
    out.backward(paddle.to_tensor(gout))
    torch.cuda.synchronize()
    assert fallback.total() == 0 and not fallback.library_counts(), (fallback.counts(), fallback.library_counts())
    af, bf = a.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    ref = (af.t() if ta else af) @ (bf.t() if tb else bf)
    ref.backward(gout.float())
    scale = K ** 0.5
    for got, want in ((out._t, ref), (x.grad._t, af.grad), (y.grad._t, bf.grad)):
        assert got.shape == want.shape
        err = (got.float() - want).abs().max().item()
        assert err <= 2e-2 * scale, err


def test_paddle_matmul_batched_left_and_bmm(monkeypatch):
    """[B, S, K] @ [K, N] flattens into the own kernels; a true bmm (per-batch right operands) runs
    on the batched own kernel (gemm4p batched mode, no fallback), with the right values"""
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    monkeypatch.setenv("PHA_GEMM_IMPL", "own")
    paddle.set_device("gpu")
    a, w = _r(3, 40, 64), _r(64, 48)
    fallback.reset()
    out = paddle.matmul(paddle.to_tensor(a), paddle.to_tensor(w))
    assert fallback.total() == 0
    torch.testing.assert_close(out._t.float(), a.float() @ w.float(), atol=0.05, rtol=0.02)
    b3 = _r(3, 64, 16)
    out = paddle.bmm(paddle.to_tensor(a), paddle.to_tensor(b3))
    assert fallback.total() == 0
    torch.testing.assert_close(out._t.float(), a.float() @ b3.float(), atol=0.05, rtol=0.02)
    lin = paddle.nn.functional.linear(paddle.to_tensor(a), paddle.to_tensor(w))
    torch.testing.assert_close(lin._t.float(), a.float() @ w.float(), atol=0.05, rtol=0.02)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 192), (1000, 2056, 640), (264, 136, 128)])
@pytest.mark.parametrize("bias", [False, True])
def test_gemm8w_nt(M, N, K, bias):
    from paddle_hackathon_amd.ops import gemm as G
    g = torch.Generator(device="cuda").manual_seed(1)
    a, bt = _r(M, K, g=g), _r(N, K, g=g)
    b = torch.randn(N, device="cuda", generator=g) if bias else None
    ref = a.float() @ bt.float().t() + (b if bias else 0)
    for relg in (2, 3, 6):
        got = G.gemm_8w(a, bt, bias=b, epi_extra=relg << 8).float()
        err = ((got - ref).abs() / (ref.abs() + 1)).max().item()
        assert err < 2e-2, (relg, err)


# ---------------------------------------------------------------------------------- quantization
def _ref_qdq(x, s, bits, round_type, dequant=True):
    bn = float(2 ** (bits - 1) - 1)
    x = x.double()
    s = s.double()
    inv = torch.where(s <= 1e-30, 1.0 / (s + 1e-6), 1.0 / s)
    if round_type == 0:
        q = torch.clamp(torch.round(bn * inv * x), -bn - 1, bn)
    else:
        v = torch.maximum(torch.minimum(x, s), -s) * bn * inv
        q = torch.sign(v) * torch.floor(v.abs() + 0.5)
    return q * s / bn if dequant else q


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("round_type", [0, 1])
def test_quant_abs_max_qdq(dtype, round_type):
    from paddle_hackathon_amd.ops import quant as Q
    g = torch.Generator(device="cuda").manual_seed(2)
    x = (torch.randn(1003, 77, device="cuda", generator=g) * 3).to(dtype)
    s = Q.abs_max(x)
    assert s.item() == x.float().abs().max().item()
    y = Q.quant_dequant(x, s, 8, round_type)
    ref = _ref_qdq(x.float(), s.float(), 8, round_type).to(dtype)
    assert y.dtype == dtype
    # rounding ties can differ by one level after the dtype's own rounding of x * bin / s
    lvl = s.item() / 127
    assert (y.float() - ref.float()).abs().max().item() <= lvl * 1.01 + 1e-6
    assert ((y.float() - ref.float()).abs() > 1e-6).float().mean().item() < 0.01
    q = Q.quant_dequant(x, s, 8, round_type, dequant=False, out_dtype=torch.float32)
    assert q.abs().max().item() <= 128 and torch.equal(q, q.round())


@pytest.mark.parametrize("shape,axis", [((64, 3, 3, 3), 0), ((96, 130), 1), ((96, 130), 0), ((4, 16, 5), 1)])
def test_quant_channel_wise(shape, axis):
    from paddle_hackathon_amd.ops import quant as Q
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(*shape, device="cuda", generator=g)
    s = Q.channel_abs_max(x, axis)
    dims = [d for d in range(x.dim()) if d != axis]
    torch.testing.assert_close(s, x.abs().amax(dim=dims), rtol=0, atol=0)
    y = Q.quant_dequant(x, s, 8, 1, quant_axis=axis)
    sh = [-1 if d == axis else 1 for d in range(x.dim())]
    ref = _ref_qdq(x, s.reshape(sh), 8, 1).float()
    torch.testing.assert_close(y, ref, rtol=0, atol=1e-5)


def test_quant_moving_average_and_ste():
    """moving-average scale recursion on device; the fake quant-dequant op's gradient is dOut"""
    from paddle_hackathon_amd.ops import quant as Q
    scale, state, accum = (torch.zeros(1, device="cuda") for _ in range(3))
    hist = []
    st = ac = 0.0
    for i in range(4):
        x = torch.randn(256, device="cuda", requires_grad=True) * (i + 1)
        x.retain_grad()
        out = Q.fake_quantize_dequantize_moving_average_abs_max(x, scale, state, accum, 8, 0.9)
        m = x.detach().abs().max().item()
        st, ac = 0.9 * st + 1, 0.9 * ac + m
        hist.append(ac / st)
        assert abs(scale.item() - hist[-1]) < 1e-5 * max(1, hist[-1])
        out.sum().backward()
        torch.testing.assert_close(x.grad, torch.ones_like(x))
