"""incubate.operators.ResNetUnit / resnet_unit and the fuse_resnet_unit pass (reference:
python/paddle/incubate/operators/resnet_unit.py, incubate/passes/fuse_resnet_unit_pass.py,
test_fuse_resnet_unit.py / test_resnet_unit_op). Oracle: conv2d + batch-statistics BN (+ add)
+ ReLU in plain fp32 torch."""
import numpy as np
import pytest
import torch

import paddle_hackathon_amd as paddle
from paddle_hackathon_amd.incubate.operators import ResNetUnit


def _bn(c):
    return (c - c.mean((0, 2, 3), keepdim=True)) / torch.sqrt(c.var((0, 2, 3), unbiased=False, keepdim=True) + 1e-5)


def _ref(u, x, z, fmt, mode, gy=None):
    def conv(t, w, s):
        if fmt == "NHWC":
            t, w = t.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2)
        return torch.nn.functional.conv2d(t, w, stride=s, padding=u._padding)
    def leaf(p):
        return p._t.detach().double().requires_grad_()

    def affine(t, sc, bi):
        return t * sc.reshape(1, -1, 1, 1) + bi.reshape(1, -1, 1, 1)
    xt, fx, sx, bx = leaf(x), leaf(u.filter_x), leaf(u.scale_x), leaf(u.bias_x)
    c = conv(xt, fx, u._stride)
    out = affine(_bn(c), sx, bx)
    grads = {"filter_x": fx, "scale_x": sx, "bias_x": bx}
    if mode == "add":
        zt = z._t.detach().double()
        out = out + (zt.permute(0, 3, 1, 2) if fmt == "NHWC" else zt)
    if mode == "short":
        fz, sz, bz = leaf(u.filter_z), leaf(u.scale_z), leaf(u.bias_z)
        grads.update(filter_z=fz, scale_z=sz, bias_z=bz)
        out = out + affine(_bn(conv(z._t.detach().double(), fz, u._stride_z)), sz, bz)
    out = torch.relu(out)
    if fmt == "NHWC":
        out = out.permute(0, 2, 3, 1)
    out.backward(torch.ones_like(out) if gy is None else gy.double().to(out.device))
    _ref.param_grads = {k: v.grad for k, v in grads.items()}
    return out, xt.grad, fx.grad, c.detach().mean((0, 2, 3))


def _check_param_grads(u, tol):
    """filter and BN scale / bias gradients against the fp64 oracle (relative, in norm)"""
    for name, ref in _ref.param_grads.items():
        g = getattr(u, name).grad
        assert g is not None, name
        r = ref.to(g._t.device)
        err = ((g._t.double() - r).norm() / r.norm().clamp_min(1e-30)).item()
        assert err < tol, (name, err)


@pytest.mark.parametrize("fmt", ["NHWC", "NCHW"])
@pytest.mark.parametrize("mode", ["plain", "add", "short"])
def test_resnet_unit_matches_conv_bn_add_relu(fmt, mode):
    paddle.seed(0)
    short = mode == "short"
    u = ResNetUnit(8, 16, 3, stride=2 if short else 1, data_format=fmt, fuse_add=mode == "add", has_shortcut=short,
                   num_channels_z=8, stride_z=2)
    shp = [2, 6, 6, 8] if fmt == "NHWC" else [2, 8, 6, 6]
    x = paddle.randn(shp)
    x.stop_gradient = False
    z = None
    if mode == "add":
        z = paddle.randn([2, 6, 6, 16] if fmt == "NHWC" else [2, 16, 6, 6])
    elif short:
        z = paddle.randn(shp)
    y = u(x, z)
    y.sum().backward()
    ref, gx, gw, mean = _ref(u, x, z, fmt, mode)
    np.testing.assert_allclose(y.numpy(), ref.detach().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(x.grad.numpy(), gx.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(u.filter_x.grad.numpy(), gw.numpy(), rtol=1e-4, atol=1e-4)
    _check_param_grads(u, 1e-5)
    # running mean moved by (1 - momentum) of the batch mean
    np.testing.assert_allclose(u.mean_x.numpy().reshape(-1), 0.1 * mean.numpy(), rtol=1e-4, atol=1e-6)
    u.eval()
    y2 = u(x, z)   # running statistics now
    assert y2.shape == y.shape
    with pytest.raises(ValueError):
        ResNetUnit(8, 16, 1, fuse_add=True)(x)


def test_fuse_resnet_unit_pass_rewrites_and_matches():
    """conv-bn-relu and conv-bn-add(conv-bn)-relu chains of a static program become two resnet_unit
    ops; the program computes the same (inference-mode BN)"""
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            x = paddle.static.data("x", [2, 8, 6, 6], "float32")
            c1, b1 = paddle.nn.Conv2D(8, 16, 3, padding=1, bias_attr=False), paddle.nn.BatchNorm2D(16)
            c2, b2 = paddle.nn.Conv2D(16, 16, 3, padding=1, bias_attr=False), paddle.nn.BatchNorm2D(16)
            cs, bs = paddle.nn.Conv2D(8, 16, 3, padding=1, bias_attr=False), paddle.nn.BatchNorm2D(16)
            for b in (b1, b2, bs):
                b.eval()
                b._mean.set_value(np.random.RandomState(1).rand(16).astype("float32"))
                b._variance.set_value(1 + np.random.RandomState(2).rand(16).astype("float32"))
            h = paddle.nn.functional.relu(b1(c1(x)))
            y = paddle.nn.functional.relu(b2(c2(h)) + bs(cs(x)))
        exe = paddle.static.Executor()
        xv = np.random.RandomState(0).randn(2, 8, 6, 6).astype("float32")
        ref, = exe.run(main, feed={"x": xv}, fetch_list=[y])
        from paddle_hackathon_amd.distributed.passes import new_pass, PassContext
        ctx = PassContext()
        new_pass("fuse_resnet_unit").apply([main], [start], ctx)
        types = [op.type.rsplit(".", 1)[-1] for op in main.global_block().ops]
        assert types == ["resnet_unit", "resnet_unit"], types
        assert ctx.get_attr("fuse_resnet_unit_count") == 2
        got, = exe.run(main, feed={"x": xv}, fetch_list=[y])
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)
    finally:
        paddle.disable_static()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["plain", "short"])
def test_resnet_unit_gpu_bf16_nhwc(mode):
    """NHWC bf16 on the MFMA convolution + fused BN-add-ReLU kernels vs the fp64 reference"""
    paddle.set_device("gpu")
    try:
        paddle.seed(0)
        short = mode == "short"
        u = ResNetUnit(64, 64, 3, stride=1, has_shortcut=short, num_channels_z=64, stride_z=1)
        for f in (u.filter_x, u.filter_z) if short else (u.filter_x,):   # bf16 filters, fp32 BN parameters
            f._t = f._t.detach().to(torch.bfloat16).requires_grad_(True)
        x = paddle.randn([4, 14, 14, 64]).astype("bfloat16")
        x.stop_gradient = False
        z = paddle.randn([4, 14, 14, 64]).astype("bfloat16") if short else None
        y = u(x, z)
        gy = torch.randn(tuple(y.shape), device="cuda")   # a random upstream gradient (a sum loss makes
        y.backward(paddle.to_tensor(gy.to(torch.bfloat16)))   # BN's backward a cancellation test)
        ref, gx, gw, _ = _ref(u, x, z, "NHWC", mode, gy.to(torch.bfloat16))
        assert y._t.dtype == torch.bfloat16
        torch.testing.assert_close(y._t.double(), ref.detach().to(y._t.device), atol=0.06, rtol=0.05)
        # the input gradient passes BN's backward (cancellations) in bf16: compare in norm. With the
        # shortcut branch the bf16-rounded residual moves the ReLU mask: the CPU torch bf16 run of the
        # same unit lands at 2.1 % from the fp64 oracle too (plain: 0.2 %)
        gxd = gx.to(y._t.device)
        assert ((x.grad._t.double() - gxd).norm() / gxd.norm()).item() < (4e-2 if short else 1e-2)
        # filter gradients (bf16 wgrad GEMM over bf16 dY) and BN scale / bias gradients (fp32)
        _check_param_grads(u, 4e-2 if short else 1.5e-2)
    finally:
        paddle.set_device("cpu")


def test_resnet_unit_saves_as_reference_op(tmp_path):
    """a program with a ResNetUnit (NHWC, reference filter layout) is written as one resnet_unit op
    with the reference slots / attributes and computes the same after loading (inference)"""
    import sys
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from test_program_desc import _strip_private
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            x = paddle.static.data("x", [2, 6, 6, 8], "float32")
            u = ResNetUnit(8, 16, 3, is_test=True)
            y = u(x)
        exe = paddle.static.Executor()
        xv = np.random.RandomState(0).randn(2, 6, 6, 8).astype("float32")
        ref, = exe.run(main, feed={"x": xv}, fetch_list=[y])
        prefix = str(tmp_path / "ru")
        paddle.static.save_inference_model(prefix, [x], [y], exe, program=main)
        desc = _strip_private(prefix + ".pdmodel")
        ops = [o for o in desc.blocks[0].ops if o.type not in ("feed", "fetch")]
        assert [o.type for o in ops] == ["resnet_unit"]
        slots = {v.parameter for v in ops[0].inputs}
        assert {"X", "FilterX", "ScaleX", "BiasX", "MeanX", "VarX"} <= slots
        attrs = {a.name for a in ops[0].attrs}
        assert {"stride", "padding", "epsilon", "data_format", "act_type", "has_shortcut"} <= attrs
        prog, _, fetches = paddle.static.load_inference_model(prefix, exe)
        got, = exe.run(prog, feed={"x": xv}, fetch_list=fetches)
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)
    finally:
        paddle.disable_static()
