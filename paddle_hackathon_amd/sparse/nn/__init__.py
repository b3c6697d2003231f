"""``paddle.sparse.nn`` layers for point-cloud style sparse 3-D conv nets (reference:
python/paddle/incubate/sparse/nn/layer/*.py). Inputs are sparse COO tensors of shape
[N, D, H, W, C] with 4 sparse dims (batch + 3 spatial) and dense channel values."""
from __future__ import annotations

import numpy as np
import torch

from ...framework.core import Tensor, _wrap
from ...nn.layer.layers import Layer
from . import functional  # noqa: F401
from . import functional as F

__all__ = ["ReLU", "ReLU6", "LeakyReLU", "Softmax", "BatchNorm", "Conv3D", "SubmConv3D", "MaxPool3D"]


class ReLU(Layer):
    def forward(self, x):
        return F.relu(x)


class ReLU6(Layer):
    def forward(self, x):
        return F.relu6(x)


class LeakyReLU(Layer):
    def __init__(self, negative_slope=0.01, name=None):
        super().__init__()
        self._slope = negative_slope

    def forward(self, x):
        return F.leaky_relu(x, self._slope)


class Softmax(Layer):
    def __init__(self, axis=-1, name=None):
        super().__init__()
        self._axis = axis

    def forward(self, x):
        return F.softmax(x, self._axis)


class BatchNorm(Layer):
    """BatchNorm over the channel values of the non-zero sites only."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format="NDHWC", use_global_stats=None, name=None):
        super().__init__()
        from ...nn import BatchNorm1D
        self._bn = BatchNorm1D(num_features, momentum=momentum, epsilon=epsilon, weight_attr=weight_attr,
                               bias_attr=bias_attr, use_global_stats=use_global_stats)

    def forward(self, x):
        c = x._t.coalesce()
        v = self._bn(_wrap(c.values()))._t
        return _wrap(torch.sparse_coo_tensor(c.indices(), v, c.shape, is_coalesced=True))


class _Conv3D(Layer):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NDHWC", subm=False, key=None):
        super().__init__()
        if groups != 1:
            raise ValueError("sparse conv3d supports groups=1 only")
        k = [kernel_size] * 3 if isinstance(kernel_size, int) else list(kernel_size)
        self._stride, self._padding, self._dilation, self._subm = stride, padding, dilation, subm
        fan_in = in_channels * int(np.prod(k))
        from ...nn import initializer as I
        self.weight = self.create_parameter(k + [in_channels, out_channels], attr=weight_attr,
                                            default_initializer=I.Normal(0.0, (2.0 / fan_in) ** 0.5))
        self.bias = None if bias_attr is False else self.create_parameter([out_channels], attr=bias_attr, is_bias=True)

    def forward(self, x):
        f = F.subm_conv3d if self._subm else F.conv3d
        return f(x, self.weight, self.bias, self._stride, self._padding, self._dilation)


class Conv3D(_Conv3D):
    def __init__(self, *a, **k):
        super().__init__(*a, subm=False, **k)


class SubmConv3D(_Conv3D):
    def __init__(self, *a, **k):
        super().__init__(*a, subm=True, **k)


class MaxPool3D(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
                 data_format="NDHWC", name=None):
        super().__init__()
        self._k, self._s, self._p = kernel_size, stride, padding

    def forward(self, x):
        return F.max_pool3d(x, self._k, self._s, self._p)
