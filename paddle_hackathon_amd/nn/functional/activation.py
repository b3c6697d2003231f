"""Activations (reference: python/paddle/nn/functional/activation.py,
phi/kernels/gpu/activation_kernel.cu, gelu_kernel.cu). GELU / bias-GELU and
softmax on HIP tensors route to our gfx950 kernels (ops/), the rest run as
PyTorch-ROCm elementwise kernels."""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _wrap, convert_dtype
from ...framework.dispatch import register_ops
from ... import ops as _ops

_w = _wrap

__all__ = ["celu", "elu", "elu_", "gelu", "glu", "gumbel_softmax", "hardshrink", "hardsigmoid",
           "hardswish", "hardtanh", "leaky_relu", "log_sigmoid", "log_softmax", "maxout", "mish",
           "prelu", "relu", "relu6", "relu_", "rrelu", "selu", "sigmoid", "silu", "softmax",
           "softmax_", "softplus", "softshrink", "softsign", "swish", "tanh", "tanh_",
           "tanhshrink", "thresholded_relu", "sigmoid_", "hard_sigmoid", "hard_swish", "relu_layer"]


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def celu(x, alpha=1.0, name=None):
    return _w(TF.celu(_t(x), alpha))


def elu(x, alpha=1.0, name=None):
    return _w(TF.elu(_t(x), alpha))


def elu_(x, alpha=1.0, name=None):
    TF.elu_(x._t, alpha)
    return x


def gelu(x, approximate=False, name=None):
    return _w(_ops.gelu(_t(x), approximate))


def glu(x, axis=-1, name=None):
    return _w(TF.glu(_t(x), axis))


def gumbel_softmax(x, temperature=1.0, hard=False, axis=-1, name=None):
    return _w(TF.gumbel_softmax(_t(x), tau=temperature, hard=hard, dim=axis))


def hardshrink(x, threshold=0.5, name=None):
    return _w(TF.hardshrink(_t(x), threshold))


def hardsigmoid(x, slope=0.1666667, offset=0.5, name=None):
    return _w(torch.clamp(_t(x) * slope + offset, 0.0, 1.0))


hard_sigmoid = hardsigmoid


def hardswish(x, name=None):
    return _w(TF.hardswish(_t(x)))


hard_swish = hardswish


def hardtanh(x, min=-1.0, max=1.0, name=None):
    return _w(TF.hardtanh(_t(x), min, max))


def leaky_relu(x, negative_slope=0.01, name=None):
    return _w(TF.leaky_relu(_t(x), negative_slope))


def log_sigmoid(x, name=None):
    return _w(TF.logsigmoid(_t(x)))


def log_softmax(x, axis=-1, dtype=None, name=None):
    t = _t(x)
    if dtype is not None:
        t = t.to(convert_dtype(dtype))
    return _w(TF.log_softmax(t, axis))


def maxout(x, groups, axis=1, name=None):
    t = _t(x)
    axis = axis % t.dim()
    shape = list(t.shape)
    c = shape[axis]
    new = shape[:axis] + [c // groups, groups] + shape[axis + 1:]
    return _w(t.reshape(new).amax(axis + 1))


def mish(x, name=None):
    return _w(TF.mish(_t(x)))


def prelu(x, weight, data_format="NCHW", name=None):
    t, w = _t(x), _t(weight)
    if w.numel() == 1:
        return _w(TF.prelu(t, w.reshape(1)))
    if data_format in ("NHWC", "NLC", "NDHWC") and t.dim() > 2:
        shape = [1] * (t.dim() - 1) + [w.numel()]
        return _w(torch.where(t > 0, t, t * w.reshape(shape)))
    return _w(TF.prelu(t, w))


def relu(x, name=None):
    return _w(torch.relu(_t(x)))


def relu_(x, name=None):
    x._t.relu_()
    return x


def relu_layer(x, name=None):
    return relu(x)


def relu6(x, name=None):
    return _w(TF.relu6(_t(x)))


def rrelu(x, lower=1.0 / 8.0, upper=1.0 / 3.0, training=True, name=None):
    return _w(TF.rrelu(_t(x), lower, upper, training))


def selu(x, scale=1.0507009873554804934193349852946, alpha=1.6732632423543772848170429916717, name=None):
    t = _t(x)
    return _w(scale * torch.where(t > 0, t, alpha * (torch.exp(t) - 1)))


def sigmoid(x, name=None):
    return _w(torch.sigmoid(_t(x)))


def sigmoid_(x, name=None):
    x._t.sigmoid_()
    return x


def silu(x, name=None):
    return _w(TF.silu(_t(x)))


def softmax(x, axis=-1, dtype=None, name=None):
    t = _t(x)
    if dtype is not None:
        t = t.to(convert_dtype(dtype))
    return _w(_ops.softmax(t, axis))


def softmax_(x, axis=-1, dtype=None, name=None):
    x._t = softmax(x, axis, dtype)._t
    return x


def softplus(x, beta=1, threshold=20, name=None):
    return _w(TF.softplus(_t(x), beta, threshold))


def softshrink(x, threshold=0.5, name=None):
    return _w(TF.softshrink(_t(x), threshold))


def softsign(x, name=None):
    return _w(TF.softsign(_t(x)))


def swish(x, name=None):
    return _w(TF.silu(_t(x)))


def tanh(x, name=None):
    return _w(torch.tanh(_t(x)))


def tanh_(x, name=None):
    x._t.tanh_()
    return x


def tanhshrink(x, name=None):
    return _w(TF.tanhshrink(_t(x)))


def thresholded_relu(x, threshold=1.0, name=None):
    t = _t(x)
    return _w(torch.where(t > threshold, t, torch.zeros_like(t)))


register_ops(globals(), __all__)
