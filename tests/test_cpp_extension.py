"""paddle.utils.cpp_extension: build a custom C++/HIP operator for gfx950, run it (host kernel
here, device kernel on the MI355X), its registered gradient op through autograd, attributes and
multiple outputs, and the setup() packaging path (reference tests: custom_op/test_custom_relu_op_jit.py,
test_custom_attrs_jit.py, test_multi_out_jit.py, test_custom_relu_op_setup.py)."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(HERE, "custom_ops", "custom_relu.cc"), os.path.join(HERE, "custom_ops", "custom_relu.hip")]


BUILD = os.path.join(HERE, "custom_ops", "_build")   # prebuilt by __graft_entry__.build() (content-stamped)


@pytest.fixture(scope="module")
def mod():
    from paddle_hackathon_amd.utils import cpp_extension
    return cpp_extension.load(name="custom_relu_test", sources=SRCS, build_directory=BUILD)


def test_custom_relu_cpu_forward_backward(mod):
    import paddle_hackathon_amd as paddle
    paddle.set_device("cpu")
    x = paddle.to_tensor(np.array([[-1.0, 2.0], [3.0, -4.0]], np.float32), stop_gradient=False)
    y = mod.custom_relu(x)
    np.testing.assert_allclose(y.numpy(), [[0, 2], [3, 0]])
    (y * paddle.to_tensor(np.array([[1.0, 2.0], [3.0, 4.0]], np.float32))).sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), [[0, 2], [3, 0]])


def test_custom_op_attrs_and_multi_out(mod):
    import paddle_hackathon_amd as paddle
    x = paddle.to_tensor(np.array([1.0, -2.0, 0.5], np.float64))
    y, cnt = mod.scale_shift(x, 2.0, 1, False, [3])
    np.testing.assert_allclose(y.numpy(), [3.0, -3.0, 2.0])
    assert int(cnt.numpy()[0]) == 2
    y2, _ = mod.scale_shift(x, scale=1.0, shift=0, negate=True, dims=[3])
    np.testing.assert_allclose(y2.numpy(), [-1.0, 2.0, -0.5])
    with pytest.raises(RuntimeError, match="dims attr"):
        mod.scale_shift(x, 1.0, 0, False, [1, 2])


def test_setup_writes_importable_module(tmp_path):
    from paddle_hackathon_amd.utils.cpp_extension import setup, CUDAExtension
    setup(name="custom_relu_pkg", ext_modules=CUDAExtension(sources=SRCS), build_directory=str(tmp_path))
    sys.path.insert(0, str(tmp_path))
    try:
        import custom_relu_pkg
        import paddle_hackathon_amd as paddle
        x = paddle.to_tensor(np.array([-1.0, 5.0], np.float32))
        np.testing.assert_allclose(custom_relu_pkg.custom_relu(x).numpy(), [0.0, 5.0])
    finally:
        sys.path.remove(str(tmp_path))


@pytest.mark.gpu
def test_custom_relu_hip_kernel_and_grad(mod):
    import paddle_hackathon_amd as paddle
    paddle.set_device("gpu:0")
    for dt in (torch.float32, torch.float16):
        xt = torch.randn(1000, 37, device="cuda", dtype=dt)
        x = paddle.to_tensor(xt, stop_gradient=False)
        y = mod.custom_relu(x)
        assert y._t.is_cuda
        torch.testing.assert_close(y._t, torch.relu(xt))
        y.sum().backward()
        torch.testing.assert_close(x.grad._t, (xt > 0).to(dt))
