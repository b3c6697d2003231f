"""Parameter initializers (reference: python/paddle/nn/initializer/*,
python/paddle/fluid/initializer.py). Initialisation draws on the HIP device
directly (no host round-trip), fan-in/out follow Paddle's layout conventions
(Linear weight is [in, out]; conv weight is [out, in/groups, *k])."""
from __future__ import annotations

import math

import numpy as np
import torch

from ..framework.core import Tensor, _unwrap

__all__ = ["Initializer", "Constant", "Normal", "TruncatedNormal", "Uniform", "XavierNormal",
           "XavierUniform", "KaimingNormal", "KaimingUniform", "Assign", "Bilinear", "Orthogonal",
           "Dirac", "calculate_gain", "set_global_initializer", "NumpyArrayInitializer",
           "MSRAInitializer", "XavierInitializer", "ConstantInitializer", "NormalInitializer",
           "UniformInitializer", "TruncatedNormalInitializer"]

_global_weight_init = None
_global_bias_init = None


def set_global_initializer(weight_init, bias_init=None):
    global _global_weight_init, _global_bias_init
    _global_weight_init = weight_init
    _global_bias_init = bias_init


def _fans(shape):
    if len(shape) == 0:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    rf = int(np.prod(shape[2:]))
    return shape[1] * rf, shape[0] * rf


def calculate_gain(nonlinearity, param=None):
    table = {"sigmoid": 1.0, "linear": 1.0, "conv1d": 1.0, "conv2d": 1.0, "conv3d": 1.0,
             "conv1d_transpose": 1.0, "conv2d_transpose": 1.0, "conv3d_transpose": 1.0,
             "tanh": 5.0 / 3, "relu": math.sqrt(2.0), "selu": 3.0 / 4}
    if nonlinearity == "leaky_relu":
        param = 0.01 if param is None else param
        return math.sqrt(2.0 / (1 + param ** 2))
    return table[nonlinearity]


class Initializer:
    def __call__(self, param, block=None):
        t = _unwrap(param)
        with torch.no_grad():
            self._init(t)
        return param

    def _init(self, t):
        raise NotImplementedError


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def _init(self, t):
        t.fill_(self.value)


class Normal(Initializer):
    def __init__(self, mean=0.0, std=1.0, name=None):
        self.mean, self.std = mean, std

    def _init(self, t):
        t.normal_(self.mean, self.std)


class TruncatedNormal(Initializer):
    def __init__(self, mean=0.0, std=1.0, name=None):
        self.mean, self.std = mean, std

    def _init(self, t):
        if t.dtype in (torch.float16, torch.bfloat16):
            tmp = torch.empty(t.shape, dtype=torch.float32, device=t.device)
            torch.nn.init.trunc_normal_(tmp, self.mean, self.std, self.mean - 2 * self.std, self.mean + 2 * self.std)
            t.copy_(tmp)
        else:
            torch.nn.init.trunc_normal_(t, self.mean, self.std, self.mean - 2 * self.std, self.mean + 2 * self.std)


class Uniform(Initializer):
    def __init__(self, low=-1.0, high=1.0, name=None):
        self.low, self.high = low, high

    def _init(self, t):
        t.uniform_(self.low, self.high)


class XavierNormal(Initializer):
    def __init__(self, fan_in=None, fan_out=None, name=None):
        self.fan_in, self.fan_out = fan_in, fan_out

    def _init(self, t):
        fi, fo = _fans(list(t.shape))
        fi = self.fan_in or fi
        fo = self.fan_out or fo
        t.normal_(0.0, math.sqrt(2.0 / (fi + fo)))


class XavierUniform(Initializer):
    def __init__(self, fan_in=None, fan_out=None, name=None):
        self.fan_in, self.fan_out = fan_in, fan_out

    def _init(self, t):
        fi, fo = _fans(list(t.shape))
        fi = self.fan_in or fi
        fo = self.fan_out or fo
        lim = math.sqrt(6.0 / (fi + fo))
        t.uniform_(-lim, lim)


class KaimingNormal(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity="relu"):
        self.fan_in, self.slope, self.nl = fan_in, negative_slope, nonlinearity

    def _init(self, t):
        fi = self.fan_in or _fans(list(t.shape))[0]
        gain = calculate_gain(self.nl, self.slope)
        t.normal_(0.0, gain / math.sqrt(fi))


class KaimingUniform(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity="relu"):
        self.fan_in, self.slope, self.nl = fan_in, negative_slope, nonlinearity

    def _init(self, t):
        fi = self.fan_in or _fans(list(t.shape))[0]
        gain = calculate_gain(self.nl, self.slope)
        lim = gain * math.sqrt(3.0 / fi)
        t.uniform_(-lim, lim)


class Assign(Initializer):
    def __init__(self, value, name=None):
        self.value = value

    def _init(self, t):
        v = self.value
        v = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
        t.copy_(v.reshape(t.shape).to(t.dtype))


NumpyArrayInitializer = Assign


class Bilinear(Initializer):
    def _init(self, t):
        shape = list(t.shape)
        size = shape[3]
        f = math.ceil(size / 2.0)
        c = (2 * f - 1 - f % 2) / (2.0 * f)
        w = torch.zeros(shape, dtype=torch.float32)
        for i in range(int(np.prod(shape))):
            x = i % size
            y = (i // size) % shape[2]
            w.view(-1)[i] = (1 - abs(x / f - c)) * (1 - abs(y / f - c))
        t.copy_(w)


class Orthogonal(Initializer):
    def __init__(self, gain=1.0, name=None):
        self.gain = gain

    def _init(self, t):
        tmp = torch.empty(t.shape, dtype=torch.float32, device=t.device)
        torch.nn.init.orthogonal_(tmp, self.gain)
        t.copy_(tmp)


class Dirac(Initializer):
    def __init__(self, groups=1, name=None):
        self.groups = groups

    def _init(self, t):
        torch.nn.init.dirac_(t, self.groups)


# fluid-era names
MSRAInitializer = KaimingNormal
XavierInitializer = XavierUniform
ConstantInitializer = Constant
NormalInitializer = Normal
UniformInitializer = Uniform
TruncatedNormalInitializer = TruncatedNormal
