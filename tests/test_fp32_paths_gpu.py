"""fp32 (Paddle's default dtype) convolutions and matmuls on the own MFMA kernels through the
three-term bf16 split (ops/conv_gemm.py split3, ops/gemm.py mm_f32; reference: the cuDNN / cuBLAS
fp32 kernels behind phi/kernels/gpudnn/conv_kernel.cu and matmul_kernel_impl.h). Oracle: fp64 torch
of the same op; the split keeps ~2^-16 relative error per product, fp32 accumulation."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("cfg", [
    # N, C, H, W, Co, k, stride, pad
    (2, 16, 14, 14, 32, 3, 1, 1),
    (2, 32, 15, 15, 16, 3, 2, 1),
    (2, 64, 8, 8, 64, 1, 2, 0),
    (2, 3, 32, 32, 24, 7, 2, 3),      # RGB stem: channels padded to 8
    (1, 8, 9, 9, 12, 3, 1, 1),        # Cout % 8 != 0
])
@pytest.mark.parametrize("fmt", ["NCHW", "NHWC"])
def test_fp32_conv2d_own_kernels(cfg, fmt):
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    N, C, H, W, Co, k, s, p = cfg
    paddle.set_device("gpu")
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda")
    w = torch.randn(Co, C, k, k, device="cuda") * (2.0 / (C * k * k)) ** 0.5
    b = torch.randn(Co, device="cuda")
    xin = x.permute(0, 2, 3, 1).contiguous() if fmt == "NHWC" else x
    px, pw, pb = paddle.to_tensor(xin), paddle.to_tensor(w), paddle.to_tensor(b)
    for t in (px, pw, pb):
        t.stop_gradient = False
    fallback.reset()
    y = paddle.nn.functional.conv2d(px, pw, pb, stride=s, padding=p, data_format=fmt)
    gy = torch.randn(tuple(y.shape), device="cuda")
    y.backward(paddle.to_tensor(gy))
    torch.cuda.synchronize()
    assert fallback.counts().get("conv2d", 0) == 0, fallback.counts()
    xd, wd, bd = (t.detach().double().requires_grad_() for t in (x, w, b))
    ref = torch.nn.functional.conv2d(xd, wd, bd, stride=s, padding=p)
    gref = gy.double().permute(0, 3, 1, 2) if fmt == "NHWC" else gy.double()
    ref.backward(gref)
    out = y._t.permute(0, 3, 1, 2) if fmt == "NHWC" else y._t
    assert y._t.dtype == torch.float32
    assert _rel(out, ref) < 2e-5
    gx = px.grad._t.permute(0, 3, 1, 2) if fmt == "NHWC" else px.grad._t
    assert _rel(gx, xd.grad) < 2e-5
    assert _rel(pw.grad._t, wd.grad) < 2e-5
    assert _rel(pb.grad._t, bd.grad) < 1e-5


def test_fp32_conv1d_runs_as_2d():
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    paddle.set_device("gpu")
    torch.manual_seed(1)
    x = torch.randn(4, 16, 50, device="cuda")
    w = torch.randn(24, 16, 5, device="cuda") * 0.1
    fallback.reset()
    y = paddle.nn.functional.conv1d(paddle.to_tensor(x), paddle.to_tensor(w), padding=2, stride=2)
    assert fallback.total() == 0, fallback.counts()
    ref = torch.nn.functional.conv1d(x.double(), w.double(), padding=2, stride=2)
    assert _rel(y._t, ref) < 2e-5


@pytest.mark.parametrize("M,K,N", [(256, 512, 384), (100, 72, 40), (7, 300, 5)])
def test_fp32_matmul_and_linear(M, K, N):
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    paddle.set_device("gpu")
    torch.manual_seed(2)
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(K, N, device="cuda")
    bias = torch.randn(N, device="cuda")
    pa, pb, pbias = paddle.to_tensor(a), paddle.to_tensor(b), paddle.to_tensor(bias)
    pa.stop_gradient = pb.stop_gradient = False
    fallback.reset()
    y = paddle.nn.functional.linear(pa, pb, pbias)
    g = torch.randn(M, N, device="cuda")
    y.backward(paddle.to_tensor(g))
    torch.cuda.synchronize()
    assert fallback.total() == 0 and not fallback.library_counts(), (fallback.counts(), fallback.library_counts())
    ad, bd = a.detach().double().requires_grad_(), b.detach().double().requires_grad_()
    ref = ad @ bd + bias.double()
    ref.backward(g.double())
    assert _rel(y._t, ref) < 2e-5
    assert _rel(pa.grad._t, ad.grad) < 2e-5
    assert _rel(pb.grad._t, bd.grad) < 2e-5
    z = paddle.matmul(pa, paddle.to_tensor(b.t().contiguous()), transpose_y=True)
    assert _rel(z._t, (a.detach().double() @ b.detach().double())) < 2e-5


def test_fp32_resnet_block_no_miopen():
    """an fp32 ResNet bottleneck (conv / BN / ReLU / residual) forward + backward without a library
    convolution"""
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    from paddle_hackathon_amd.vision.models.resnet import BottleneckBlock
    paddle.set_device("gpu")
    paddle.seed(0)
    blk = BottleneckBlock(64, 16, stride=1)
    x = paddle.randn([4, 64, 16, 16])
    x.stop_gradient = False
    fallback.reset()
    y = blk(x)
    y.sum().backward()
    torch.cuda.synchronize()
    assert fallback.counts().get("conv2d", 0) == 0, fallback.counts()
    assert y._t.dtype == torch.float32 and torch.isfinite(x.grad._t).all()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("fmt", ["NCDHW", "NDHWC"])
def test_conv3d_own_kernels(dtype, fmt):
    """3-D convolution as per-depth-tap 2-D convolutions on the own kernels (forward + backward)"""
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    paddle.set_device("gpu")
    torch.manual_seed(5)
    x = torch.randn(2, 8, 6, 10, 10, device="cuda")
    w = torch.randn(16, 8, 3, 3, 3, device="cuda") * 0.1
    b = torch.randn(16, device="cuda")
    xin = x.permute(0, 2, 3, 4, 1).contiguous() if fmt == "NDHWC" else x
    px, pw, pb = (paddle.to_tensor(v.to(dtype)) for v in (xin, w, b))
    for t in (px, pw, pb):
        t.stop_gradient = False
    fallback.reset()
    y = paddle.nn.functional.conv3d(px, pw, pb, stride=[2, 1, 1], padding=1, data_format=fmt)
    y.astype("float32").sum().backward()
    assert fallback.counts().get("conv3d", 0) == 0, fallback.counts()
    xd, wd = x.detach().to(dtype).double().requires_grad_(), w.detach().to(dtype).double().requires_grad_()
    ref = torch.nn.functional.conv3d(xd, wd, b.to(dtype).double(), stride=[2, 1, 1], padding=1)
    ref.sum().backward()
    out = y._t.permute(0, 4, 1, 2, 3) if fmt == "NDHWC" else y._t
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert _rel(out, ref) < tol
    gx = px.grad._t.permute(0, 4, 1, 2, 3) if fmt == "NDHWC" else px.grad._t
    assert _rel(gx, xd.grad) < tol
    assert _rel(pw.grad._t, wd.grad) < tol


@pytest.mark.gpu
@pytest.mark.parametrize("shape,dim,order", [((4, 6, 6, 24), 3, "hhl"), ((64, 40), 0, "hlh"), ((3, 5, 16), 1, "lhl")])
def test_split3_kernel_matches_torch(shape, dim, order):
    """csrc/kernels/split.hip: the one-pass fp32 -> [hi | lo] bf16 split equals the torch expression
    bit for bit (round-to-nearest-even for both terms)"""
    from paddle_hackathon_amd.ops import conv_gemm
    torch.manual_seed(0)
    t = torch.randn(*shape, device="cuda") * 100
    got = conv_gemm.split3(t, dim, order)
    hi = t.to(torch.bfloat16)
    lo = (t - hi.float()).to(torch.bfloat16)
    ref = torch.cat([hi if c == "h" else lo for c in order], dim)
    assert got.shape == ref.shape and torch.equal(got.view(torch.int16), ref.view(torch.int16))


def test_fp32_split_extremes():
    """the split of values past the bf16 range and of non-finite values: finite inputs
    near FLT_MAX stay finite (hi truncated, lo exact) and an inf / NaN input gives a non-finite
    product wherever the fp64 product is non-finite (what AMP overflow checks read)"""
    from paddle_hackathon_amd.ops import conv_gemm, gemm
    torch.manual_seed(3)
    t = torch.tensor([1.0, 3.39e38, -3.39e38, float("inf"), float("-inf"), float("nan"), 1e-3, 123.456] * 2,
                     device="cuda")
    s = conv_gemm.split3(t, 0, "hlh").float()   # three parts along dim 0: hi, lo, hi
    hi, lo = s[:16], s[16:32]
    torch.testing.assert_close(s[32:], hi, rtol=0, atol=0, equal_nan=True)
    fin = torch.isfinite(t)
    assert torch.isfinite(hi[fin]).all() and torch.isfinite(lo).all()
    rel = ((hi[fin].double() + lo[fin].double() - t[fin].double()).abs() / t[fin].double().abs()).max().item()
    assert rel < 2e-5
    assert torch.isinf(hi[3]) and torch.isinf(hi[4]) and torch.isnan(hi[5])
    # a GEMM with large finite entries: finite, ~2^-16 relative to fp64
    a = torch.randn(64, 128, device="cuda")
    b = torch.randn(128, 64, device="cuda")
    a[0, :4] = 3e37
    y = gemm.mm_f32(a, b)
    ref = a.double() @ b.double()
    assert torch.isfinite(y).all() and _rel(y, ref) < 2e-5
    # an inf row: non-finite exactly where fp64 is non-finite, finite rows unchanged
    a2 = a.clone()
    a2[5, 7] = float("inf")
    y2 = gemm.mm_f32(a2, b)
    ref2 = a2.double() @ b.double()
    assert torch.equal(torch.isfinite(y2), torch.isfinite(ref2))
