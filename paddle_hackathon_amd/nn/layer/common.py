"""Common layers (reference: python/paddle/nn/layer/common.py, activation.py, distance.py, vision.py)."""
from __future__ import annotations

import numpy as np

from ...framework.core import Tensor
from ...framework.param_attr import ParamAttr
from .. import functional as F
from .. import initializer as I
from .layers import Layer

__all__ = ["Linear", "Embedding", "Dropout", "Dropout2D", "Dropout3D", "AlphaDropout", "Flatten", "Identity",
           "Pad1D", "Pad2D", "Pad3D", "ZeroPad2D", "Upsample", "UpsamplingNearest2D", "UpsamplingBilinear2D",
           "Bilinear", "CosineSimilarity", "Unfold", "Fold", "PixelShuffle", "PixelUnshuffle", "ChannelShuffle",
           "PairwiseDistance", "ReLU", "ReLU6", "LeakyReLU", "PReLU", "RReLU", "ELU", "CELU", "SELU", "GELU",
           "Sigmoid", "Hardsigmoid", "Hardswish", "Hardtanh", "Hardshrink", "Softshrink", "Tanhshrink", "Tanh",
           "Softplus", "Softsign", "Swish", "Silu", "Mish", "LogSigmoid", "Softmax", "Softmax2D", "LogSoftmax",
           "Maxout", "ThresholdedReLU", "GLU"]


class Linear(Layer):
    """y = xW + b, W: [in_features, out_features] (Paddle layout)."""

    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self._dtype = self._dtype
        self.weight = self.create_parameter([in_features, out_features], attr=weight_attr)
        self.bias = self.create_parameter([out_features], attr=bias_attr, is_bias=True)
        self.in_features, self.out_features = in_features, out_features
        self.name = name

    def forward(self, input):
        return F.linear(input, self.weight, self.bias)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, dtype={self._dtype}"


class Embedding(Layer):
    def __init__(self, num_embeddings, embedding_dim, padding_idx=None, sparse=False, weight_attr=None, name=None):
        super().__init__()
        self._num_embeddings, self._embedding_dim = num_embeddings, embedding_dim
        if padding_idx is not None and padding_idx < 0:
            padding_idx += num_embeddings
        self._padding_idx = padding_idx
        self._sparse = sparse
        self.weight = self.create_parameter([num_embeddings, embedding_dim], attr=weight_attr,
                                            default_initializer=I.XavierUniform())
        if padding_idx is not None:
            import torch
            with torch.no_grad():
                self.weight._t[padding_idx].zero_()

    def forward(self, x):
        return F.embedding(x, self.weight, self._padding_idx, self._sparse)

    def extra_repr(self):
        return f"{self._num_embeddings}, {self._embedding_dim}"


class Dropout(Layer):
    def __init__(self, p=0.5, axis=None, mode="upscale_in_train", name=None):
        super().__init__()
        self.p, self.axis, self.mode = p, axis, mode

    def forward(self, input):
        return F.dropout(input, self.p, self.axis, self.training, self.mode)

    def extra_repr(self):
        return f"p={self.p}, axis={self.axis}, mode={self.mode}"


class Dropout2D(Layer):
    def __init__(self, p=0.5, data_format="NCHW", name=None):
        super().__init__()
        self.p, self.data_format = p, data_format

    def forward(self, input):
        return F.dropout2d(input, self.p, self.training, self.data_format)


class Dropout3D(Layer):
    def __init__(self, p=0.5, data_format="NCDHW", name=None):
        super().__init__()
        self.p, self.data_format = p, data_format

    def forward(self, input):
        return F.dropout3d(input, self.p, self.training, self.data_format)


class AlphaDropout(Layer):
    def __init__(self, p=0.5, name=None):
        super().__init__()
        self.p = p

    def forward(self, input):
        return F.alpha_dropout(input, self.p, self.training)


class Flatten(Layer):
    def __init__(self, start_axis=1, stop_axis=-1):
        super().__init__()
        self.start_axis, self.stop_axis = start_axis, stop_axis

    def forward(self, input):
        from ...tensor import flatten
        return flatten(input, self.start_axis, self.stop_axis)


class Identity(Layer):
    def __init__(self, *args, **kwargs):
        super().__init__()

    def forward(self, input):
        return input


class _PadNd(Layer):
    _n = 2
    _default_fmt = "NCHW"

    def __init__(self, padding, mode="constant", value=0.0, data_format=None, name=None):
        super().__init__()
        if isinstance(padding, int):
            padding = [padding] * (2 * self._n)
        self._pad, self._mode, self._value = padding, mode, value
        self._data_format = data_format or self._default_fmt

    def forward(self, x):
        return F.pad(x, self._pad, self._mode, self._value, self._data_format)


class Pad1D(_PadNd):
    _n, _default_fmt = 1, "NCL"


class Pad2D(_PadNd):
    _n, _default_fmt = 2, "NCHW"


class Pad3D(_PadNd):
    _n, _default_fmt = 3, "NCDHW"


class ZeroPad2D(_PadNd):
    _n, _default_fmt = 2, "NCHW"

    def __init__(self, padding, data_format="NCHW", name=None):
        super().__init__(padding, "constant", 0.0, data_format)


class Upsample(Layer):
    def __init__(self, size=None, scale_factor=None, mode="nearest", align_corners=False, align_mode=0,
                 data_format="NCHW", name=None):
        super().__init__()
        self.size, self.scale_factor, self.mode = size, scale_factor, mode
        self.align_corners, self.align_mode, self.data_format = align_corners, align_mode, data_format

    def forward(self, x):
        return F.interpolate(x, self.size, self.scale_factor, self.mode, self.align_corners, self.align_mode, self.data_format)


class UpsamplingNearest2D(Upsample):
    def __init__(self, size=None, scale_factor=None, data_format="NCHW", name=None):
        super().__init__(size, scale_factor, "nearest", False, 0, data_format)


class UpsamplingBilinear2D(Upsample):
    def __init__(self, size=None, scale_factor=None, data_format="NCHW", name=None):
        super().__init__(size, scale_factor, "bilinear", True, 0, data_format)


class Bilinear(Layer):
    def __init__(self, in1_features, in2_features, out_features, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self.weight = self.create_parameter([out_features, in1_features, in2_features], attr=weight_attr)
        self.bias = self.create_parameter([1, out_features], attr=bias_attr, is_bias=True)

    def forward(self, x1, x2):
        return F.bilinear(x1, x2, self.weight, self.bias)


class CosineSimilarity(Layer):
    def __init__(self, axis=1, eps=1e-8):
        super().__init__()
        self.axis, self.eps = axis, eps

    def forward(self, x1, x2):
        return F.cosine_similarity(x1, x2, self.axis, self.eps)


class PairwiseDistance(Layer):
    def __init__(self, p=2.0, epsilon=1e-6, keepdim=False, name=None):
        super().__init__()
        self.p, self.eps, self.keepdim = p, epsilon, keepdim

    def forward(self, x, y):
        return F.pairwise_distance(x, y, self.p, self.eps, self.keepdim)


class Unfold(Layer):
    def __init__(self, kernel_sizes, dilations=1, paddings=0, strides=1, name=None):
        super().__init__()
        self.args = (kernel_sizes, strides, paddings, dilations)

    def forward(self, input):
        k, s, p, d = self.args
        return F.unfold(input, k, s, p, d)


class Fold(Layer):
    def __init__(self, output_sizes, kernel_sizes, dilations=1, paddings=0, strides=1, name=None):
        super().__init__()
        self.args = (output_sizes, kernel_sizes, strides, paddings, dilations)

    def forward(self, input):
        o, k, s, p, d = self.args
        return F.fold(input, o, k, s, p, d)


class PixelShuffle(Layer):
    def __init__(self, upscale_factor, data_format="NCHW", name=None):
        super().__init__()
        self.f, self.df = upscale_factor, data_format

    def forward(self, x):
        return F.pixel_shuffle(x, self.f, self.df)


class PixelUnshuffle(Layer):
    def __init__(self, downscale_factor, data_format="NCHW", name=None):
        super().__init__()
        self.f, self.df = downscale_factor, data_format

    def forward(self, x):
        return F.pixel_unshuffle(x, self.f, self.df)


class ChannelShuffle(Layer):
    def __init__(self, groups, data_format="NCHW", name=None):
        super().__init__()
        self.g, self.df = groups, data_format

    def forward(self, x):
        return F.channel_shuffle(x, self.g, self.df)


# ---------------------------------------------------------------------------- activations
def _act(name, fn, argnames=(), defaults=()):
    def __init__(self, *args, **kwargs):
        Layer.__init__(self)
        vals = dict(zip(argnames, defaults))
        for k, v in zip(argnames, args):
            vals[k] = v
        for k, v in kwargs.items():
            if k != "name":
                vals[k] = v
        self._args = vals

    def forward(self, x):
        return fn(x, **self._args)

    def extra_repr(self):
        return ", ".join(f"{k}={v}" for k, v in self._args.items())

    return type(name, (Layer,), {"__init__": __init__, "forward": forward, "extra_repr": extra_repr})


ReLU = _act("ReLU", F.relu)
ReLU6 = _act("ReLU6", F.relu6)
LeakyReLU = _act("LeakyReLU", F.leaky_relu, ("negative_slope",), (0.01,))
ELU = _act("ELU", F.elu, ("alpha",), (1.0,))
CELU = _act("CELU", F.celu, ("alpha",), (1.0,))
SELU = _act("SELU", F.selu, ("scale", "alpha"), (1.0507009873554804934193349852946, 1.6732632423543772848170429916717))
GELU = _act("GELU", F.gelu, ("approximate",), (False,))
Sigmoid = _act("Sigmoid", F.sigmoid)
Hardsigmoid = _act("Hardsigmoid", F.hardsigmoid)
Hardswish = _act("Hardswish", F.hardswish)
Hardtanh = _act("Hardtanh", F.hardtanh, ("min", "max"), (-1.0, 1.0))
Hardshrink = _act("Hardshrink", F.hardshrink, ("threshold",), (0.5,))
Softshrink = _act("Softshrink", F.softshrink, ("threshold",), (0.5,))
Tanhshrink = _act("Tanhshrink", F.tanhshrink)
Tanh = _act("Tanh", F.tanh)
Softplus = _act("Softplus", F.softplus, ("beta", "threshold"), (1, 20))
Softsign = _act("Softsign", F.softsign)
Swish = _act("Swish", F.swish)
Silu = _act("Silu", F.silu)
Mish = _act("Mish", F.mish)
LogSigmoid = _act("LogSigmoid", F.log_sigmoid)
Softmax = _act("Softmax", F.softmax, ("axis",), (-1,))
LogSoftmax = _act("LogSoftmax", F.log_softmax, ("axis",), (-1,))
Maxout = _act("Maxout", F.maxout, ("groups", "axis"), (None, 1))
ThresholdedReLU = _act("ThresholdedReLU", F.thresholded_relu, ("threshold",), (1.0,))
GLU = _act("GLU", F.glu, ("axis",), (-1,))


class Softmax2D(Layer):
    def __init__(self, name=None):
        super().__init__()

    def forward(self, x):
        return F.softmax(x, axis=-3)


class RReLU(Layer):
    def __init__(self, lower=1.0 / 8.0, upper=1.0 / 3.0, name=None):
        super().__init__()
        self.lower, self.upper = lower, upper

    def forward(self, x):
        return F.rrelu(x, self.lower, self.upper, self.training)


class PReLU(Layer):
    def __init__(self, num_parameters=1, init=0.25, weight_attr=None, data_format="NCHW", name=None):
        super().__init__()
        self._data_format = data_format
        self.weight = self.create_parameter([num_parameters], attr=weight_attr, default_initializer=I.Constant(init))

    def forward(self, x):
        return F.prelu(x, self.weight, self._data_format)
