"""Own convolution coverage beyond dense NHWC bf16 (GPU only): grouped / depthwise / dilated +
strided convolutions on the direct HIP kernels (ops/grouped_conv.py), NCHW networks kept in
channels-last memory on the own kernels, checked against plain PyTorch fp32 convolutions, and whole
zoo models (ResNet-50 NCHW default, MobileNetV2, ResNeXt, ShuffleNetV2) recording no conv fallback."""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _native():
    from paddle_hackathon_amd.ops import _lib
    assert _lib.native_available(), "libpha_kernels.so must be loaded on a GPU run"
    yield


def _close(a, r, dt, what):
    tol = {torch.float32: 1e-4, torch.bfloat16: 3e-2, torch.float16: 4e-3}[dt]
    err = (a.float() - r).abs().max().item()
    assert err <= tol * max(1.0, r.abs().max().item()), (what, err, r.abs().max().item())


# (N, C, H, W, CO, k, stride, pad, dil, groups)
CASES = [
    (4, 32, 17, 15, 32, 3, 1, 1, 1, 32),      # depthwise 3x3
    (4, 64, 16, 16, 64, 3, 2, 1, 1, 64),      # depthwise stride 2
    (2, 32, 12, 12, 64, 5, 1, 2, 1, 32),      # channel multiplier 2 (ANY mode)
    (2, 128, 14, 14, 128, 3, 1, 1, 1, 32),    # ResNeXt 32 x 4d (cig = cog = 4)
    (2, 64, 10, 10, 128, 3, 1, 1, 1, 4),      # groups 4, cig 16, cog 32 (vector modes)
    (2, 16, 20, 20, 24, 3, 2, 2, 2, 1),       # dense dilated + strided
    (2, 8, 9, 9, 21, 1, 1, 0, 1, 1),          # dense, 21 output channels (padded)
    (2, 3, 16, 16, 8, 3, 2, 2, 2, 1),         # dense, 3 input channels, dilated + strided
    (2, 58, 9, 9, 58, 3, 2, 1, 1, 58),        # depthwise, 58 channels (ShuffleNetV2, padded)
    (2, 16, 10, 10, 16, 3, 1, 1, 1, 8),       # cig = cog = 2 (GRP2)
    (2, 24, 10, 10, 32, 3, 1, 1, 1, 2),       # cig 12, cog 16 (scalar-input SAME / ANY)
    (2, 256, 7, 7, 256, 3, 1, 1, 1, 32),      # ResNeXt late stage (cig = cog = 8)
]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("case", CASES)
def test_direct_conv_fwd_bwd(case, dt):
    from paddle_hackathon_amd.ops import grouped_conv as gc
    N, C, H, W, CO, k, s, p, d, g = case
    if dt == torch.float32 and g == 1:
        pytest.skip("dense fp32 convolutions stay on MIOpen")
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device="cuda").to(dt)
    w = (torch.randn(CO, C // g, k, k, device="cuda") / (C // g * k * k) ** 0.5).to(dt)
    b = torch.randn(CO, device="cuda").to(dt)
    xr, wr, br = (t.float().detach().requires_grad_(True) for t in (x, w, b))
    ref = TF.conv2d(xr.permute(0, 3, 1, 2), wr, br, s, p, d, g).permute(0, 2, 3, 1)
    xa, wa, ba = (t.detach().requires_grad_(True) for t in (x, w, b))
    y = gc.conv2d_nhwc(xa, wa, ba, (s, s), (p, p), (d, d), g)
    assert y.shape == ref.shape
    _close(y, ref, dt, "fwd")
    gy = torch.randn_like(ref)
    ref.backward(gy)
    y.backward(gy.to(dt))
    _close(xa.grad, xr.grad, dt, "dx")
    _close(wa.grad, wr.grad, dt, "dw")
    _close(ba.grad, br.grad, dt, "db")


@pytest.mark.parametrize("fmt", ["NCHW", "NHWC"])
@pytest.mark.parametrize("groups,k,stride,dil,padding", [(1, 3, 1, 1, 1), (1, 3, 2, 1, "SAME"), (8, 3, 1, 1, 1),
                                                        (32, 3, 2, 1, 1), (1, 3, 2, 2, 2)])
def test_conv2d_dispatch_own_kernels(fmt, groups, k, stride, dil, padding):
    """paddle.nn.functional.conv2d in either data format runs on the own kernels (no fallback) and
    matches fp32; an NCHW result is NHWC in memory, and BN / max-pool on it run the NHWC kernels"""
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    from paddle_hackathon_amd.nn.functional.conv import nhwc_view
    paddle.set_device("gpu")
    torch.manual_seed(0)
    N, C, H, W, CO = 2, 32, 15, 16, 64
    x = torch.randn(N, C, H, W, device="cuda").bfloat16()
    w = (torch.randn(CO, C // groups, k, k, device="cuda") / (C // groups * k * k) ** 0.5).bfloat16()
    xin = x if fmt == "NCHW" else x.permute(0, 2, 3, 1).contiguous()
    fallback.reset()
    y = paddle.nn.functional.conv2d(paddle.to_tensor(xin), paddle.to_tensor(w), stride=stride, padding=padding,
                                    dilation=dil, groups=groups, data_format=fmt)
    assert fallback.counts().get("conv2d", 0) == 0, fallback.counts()
    yt = y._t if fmt == "NCHW" else y._t.permute(0, 3, 1, 2)
    if padding == "SAME":
        oh, ow = -(-H // stride), -(-W // stride)
        ph, pw = max((oh - 1) * stride + k - H, 0), max((ow - 1) * stride + k - W, 0)
        xp = TF.pad(x.float(), [pw // 2, pw - pw // 2, ph // 2, ph - ph // 2])
        ref = TF.conv2d(xp, w.float(), None, stride, 0, dil, groups)
    else:
        ref = TF.conv2d(x.float(), w.float(), None, stride, padding, dil, groups)
    _close(yt, ref, torch.bfloat16, "conv2d")
    if fmt == "NCHW":
        assert nhwc_view(y._t) is not None, "NCHW conv output is channels-last in memory"
        rm, rv = torch.zeros(CO, device="cuda"), torch.ones(CO, device="cuda")
        gam, bet = torch.rand(CO, device="cuda") + 0.5, torch.randn(CO, device="cuda")
        bn = paddle.nn.functional.batch_norm(y, paddle.to_tensor(rm.clone()), paddle.to_tensor(rv.clone()),
                                             paddle.to_tensor(gam), paddle.to_tensor(bet), training=True)
        bnr = TF.batch_norm(yt.float(), rm.clone(), rv.clone(), gam, bet, True, 0.1, 1e-5)
        _close(bn._t, bnr, torch.bfloat16, "batch_norm")
        z = paddle.nn.functional.max_pool2d(y, 3, 2, 1)
        zr = TF.max_pool2d(ref, 3, 2, 1)
        _close(z._t, zr, torch.bfloat16, "maxpool")


@pytest.mark.parametrize("s2d", ["1", "0"])
@pytest.mark.parametrize("H,W,k,s,p", [(32, 32, 7, 2, 3), (33, 30, 7, 2, 3), (20, 20, 3, 2, 1)])
def test_rgb_stem_conv_space_to_depth(monkeypatch, s2d, H, W, k, s, p):
    """the RGB stem (3 channels, stride 2) through paddle conv2d on the own kernels, as the stride-1
    convolution of its space-to-depth image (PHA_CONV_S2D=1, default) or padded to 8 channels:
    output, dx and dw match fp32"""
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    monkeypatch.setenv("PHA_CONV_S2D", s2d)
    paddle.set_device("gpu")
    torch.manual_seed(0)
    x = torch.randn(4, H, W, 3, device="cuda").bfloat16()
    w = (torch.randn(64, 3, k, k, device="cuda") / (3 * k * k) ** 0.5).bfloat16()
    xr, wr = (t.float().detach().requires_grad_(True) for t in (x, w))
    ref = TF.conv2d(xr.permute(0, 3, 1, 2), wr, None, s, p).permute(0, 2, 3, 1)
    xa, wa = paddle.to_tensor(x), paddle.to_tensor(w)
    xa.stop_gradient = False
    wa.stop_gradient = False
    fallback.reset()
    y = paddle.nn.functional.conv2d(xa, wa, stride=s, padding=p, data_format="NHWC")
    assert fallback.counts().get("conv2d", 0) == 0, fallback.counts()
    assert tuple(y.shape) == tuple(ref.shape)
    _close(y._t, ref, torch.bfloat16, "fwd")
    gy = torch.randn_like(ref)
    ref.backward(gy)
    (y * paddle.to_tensor(gy.bfloat16())).sum().backward()
    _close(xa.grad._t, xr.grad, torch.bfloat16, "dx")
    _close(wa.grad._t, wr.grad, torch.bfloat16, "dw")


def _no_conv_fallback_step(model, x, y):
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    model = paddle.amp.decorate(model, level="O2", dtype="bfloat16")
    opt = paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=model.parameters(),
                                    multi_precision=True)
    fallback.reset()
    for _ in range(2):
        with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
            loss = paddle.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad(set_to_zero=False)
    torch.cuda.synchronize()
    assert torch.isfinite(torch.tensor(float(loss.item())))
    return fallback.counts()


@pytest.mark.parametrize("name", ["resnet50", "mobilenet_v2", "resnext50_32x4d", "shufflenet_v2_x1_0"])
def test_zoo_models_nchw_no_conv_fallback(name):
    """the zoo models in their default NCHW format train on the own conv kernels only"""
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.vision import models
    paddle.set_device("gpu")
    paddle.seed(0)
    model = getattr(models, name)()
    x = paddle.to_tensor(torch.randn(4, 3, 64, 64, device="cuda").bfloat16())
    y = paddle.to_tensor(torch.randint(0, 1000, (4,), device="cuda"))
    counts = _no_conv_fallback_step(model, x, y)
    assert counts.get("conv2d", 0) == 0, counts


# (N, Cin, H, W, Cout, k, stride, pad, out_pad, dil, groups, dtype)
TCASES = [
    (2, 32, 8, 9, 16, 4, 2, 1, 0, 1, 1, torch.bfloat16),    # DCGAN-style 4x4 stride-2 upsample
    (2, 16, 7, 7, 32, 3, 2, 1, 1, 1, 1, torch.bfloat16),    # output_padding 1
    (2, 24, 6, 6, 40, 3, 1, 1, 0, 1, 1, torch.float16),     # stride 1
    (2, 32, 6, 6, 32, 3, 2, 2, 1, 2, 1, torch.bfloat16),    # dilated + strided (direct)
    (2, 64, 5, 5, 64, 3, 2, 1, 1, 1, 64, torch.bfloat16),   # depthwise (direct)
    (2, 32, 6, 6, 64, 3, 1, 1, 0, 1, 4, torch.float32),     # grouped fp32 (direct)
]


@pytest.mark.parametrize("fmt", ["NCHW", "NHWC"])
@pytest.mark.parametrize("case", TCASES)
def test_conv2d_transpose_own_kernels(case, fmt):
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    N, Cin, H, W, Cout, k, s, p, op, d, g, dt = case
    paddle.set_device("gpu")
    torch.manual_seed(0)
    x = torch.randn(N, Cin, H, W, device="cuda").to(dt)
    w = (torch.randn(Cin, Cout // g, k, k, device="cuda") / (Cin * k * k / s / s) ** 0.5).to(dt)
    b = torch.randn(Cout, device="cuda").to(dt)
    xr, wr, br = (t.float().detach().requires_grad_(True) for t in (x, w, b))
    ref = TF.conv_transpose2d(xr, wr, br, s, p, op, g, d)
    xin = x if fmt == "NCHW" else x.permute(0, 2, 3, 1).contiguous()
    xa, wa, ba = (paddle.to_tensor(t) for t in (xin, w, b))
    for t in (xa, wa, ba):
        t.stop_gradient = False
    fallback.reset()
    y = paddle.nn.functional.conv2d_transpose(xa, wa, ba, stride=s, padding=p, output_padding=op, dilation=d,
                                              groups=g, data_format=fmt)
    assert fallback.counts().get("conv2d", 0) == 0, fallback.counts()
    yt = y._t if fmt == "NCHW" else y._t.permute(0, 3, 1, 2)
    assert yt.shape == ref.shape
    _close(yt, ref, dt, "fwd")
    gy = torch.randn_like(ref)
    ref.backward(gy)
    gin = gy.to(dt) if fmt == "NCHW" else gy.to(dt).permute(0, 2, 3, 1).contiguous()
    y._t.backward(gin)
    gx = xa._t.grad if fmt == "NCHW" else xa._t.grad.permute(0, 3, 1, 2)
    _close(gx, xr.grad, dt, "dx")
    _close(wa._t.grad, wr.grad, dt, "dw")
    _close(ba._t.grad, br.grad, dt, "db")


@pytest.mark.parametrize("cfg", [
    # N, C, H, W, Co, groups, k, stride, pad
    (4, 128, 14, 14, 128, 32, 3, 1, 1),    # ResNeXt 32x4d stage 1 (cig 4: groups merged in pairs)
    (4, 256, 14, 14, 256, 32, 3, 2, 1),    # cig 8, strided
    (2, 512, 7, 7, 512, 32, 3, 1, 1),      # cig 16
    (2, 64, 9, 9, 128, 2, 3, 1, 1),        # few wide groups
])
def test_grouped_conv_mfma(cfg):
    """grouped convolutions on the grouped implicit GEMM (forward, dgrad, wgrad) vs fp32 torch"""
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import fallback
    N, C, H, W, Co, g, k, s, p = cfg
    paddle.set_device("gpu")
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Co, C // g, k, k, device="cuda") * (2.0 / (C // g * k * k)) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Co, device="cuda").to(torch.bfloat16)
    px, pw, pb = paddle.to_tensor(x), paddle.to_tensor(w), paddle.to_tensor(b)
    for t in (px, pw, pb):
        t.stop_gradient = False
    fallback.reset()
    y = paddle.nn.functional.conv2d(px, pw, pb, stride=s, padding=p, groups=g, data_format="NHWC")
    gy = torch.randn(tuple(y.shape), device="cuda").to(torch.bfloat16)
    y.backward(paddle.to_tensor(gy))
    torch.cuda.synchronize()
    assert fallback.total() == 0, fallback.counts()
    xd, wd, bd = (t.detach().float().requires_grad_() for t in (x, w, b))
    ref = torch.nn.functional.conv2d(xd.permute(0, 3, 1, 2), wd, bd, stride=s, padding=p, groups=g).permute(0, 2, 3, 1)
    ref.backward(gy.float())

    def rel(a, r):
        return ((a.float() - r).norm() / r.norm()).item()
    assert rel(y._t, ref) < 1e-2
    assert rel(px.grad._t, xd.grad) < 1e-2
    assert rel(pw.grad._t, wd.grad) < 1e-2
    assert rel(pb.grad._t, bd.grad) < 1e-2
