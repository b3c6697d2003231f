"""Conv / norm / pooling layers (reference: python/paddle/nn/layer/{conv,norm,pooling}.py)."""
from __future__ import annotations

import numpy as np
import torch

from ...framework import core as _core
from ...framework.core import Tensor, _wrap
from .. import functional as F
from .. import initializer as I
from .layers import Layer

__all__ = ["Conv1D", "Conv2D", "Conv3D", "Conv1DTranspose", "Conv2DTranspose", "Conv3DTranspose",
           "BatchNorm", "BatchNorm1D", "BatchNorm2D", "BatchNorm3D", "SyncBatchNorm", "LayerNorm", "GroupNorm",
           "InstanceNorm1D", "InstanceNorm2D", "InstanceNorm3D", "LocalResponseNorm", "SpectralNorm", "RMSNorm",
           "AvgPool1D", "AvgPool2D", "AvgPool3D", "MaxPool1D", "MaxPool2D", "MaxPool3D", "AdaptiveAvgPool1D",
           "AdaptiveAvgPool2D", "AdaptiveAvgPool3D", "AdaptiveMaxPool1D", "AdaptiveMaxPool2D", "AdaptiveMaxPool3D",
           "MaxUnPool1D", "MaxUnPool2D", "MaxUnPool3D"]


def _ntuple(v, n):
    return list(v) if isinstance(v, (list, tuple)) else [v] * n


class _ConvNd(Layer):
    _n = 2
    _transpose = False

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, dilation=1,
                 groups=1, padding_mode="zeros", weight_attr=None, bias_attr=None, data_format=None):
        super().__init__()
        n = self._n
        self._in_channels, self._out_channels = in_channels, out_channels
        self._kernel_size = _ntuple(kernel_size, n)
        self._stride, self._padding, self._dilation = stride, padding, dilation
        self._output_padding = output_padding
        self._groups = groups
        self._padding_mode = padding_mode
        self._data_format = data_format or {1: "NCL", 2: "NCHW", 3: "NCDHW"}[n]
        if self._transpose:
            shape = [in_channels, out_channels // groups] + self._kernel_size
        else:
            shape = [out_channels, in_channels // groups] + self._kernel_size
        fan_in = (in_channels // groups) * int(np.prod(self._kernel_size))
        std = (2.0 / fan_in) ** 0.5
        self.weight = self.create_parameter(shape, attr=weight_attr, default_initializer=I.Normal(0.0, std))
        self.bias = self.create_parameter([out_channels], attr=bias_attr, is_bias=True)

    def _pad_input(self, x):
        if self._padding_mode != "zeros" and not self._transpose:
            p = _ntuple(self._padding, self._n) if not isinstance(self._padding, str) else [0] * self._n
            pads = []
            for v in reversed(p):
                pads += [v, v]
            mode = {"reflect": "reflect", "replicate": "replicate", "circular": "circular"}[self._padding_mode]
            return F.pad(x, pads, mode=mode, data_format=self._data_format), 0
        return x, self._padding

    def forward(self, x, output_size=None):
        if self._transpose:
            f = {1: F.conv1d_transpose, 2: F.conv2d_transpose, 3: F.conv3d_transpose}[self._n]
            if self._n == 2:
                return f(x, self.weight, self.bias, self._stride, self._padding, self._output_padding, self._dilation,
                         self._groups, output_size, self._data_format)
            return f(x, self.weight, self.bias, self._stride, self._padding, self._output_padding, self._groups,
                     self._dilation, output_size, self._data_format)
        x, pad = self._pad_input(x)
        f = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}[self._n]
        return f(x, self.weight, self.bias, self._stride, pad, self._dilation, self._groups, self._data_format)

    def extra_repr(self):
        return (f"{self._in_channels}, {self._out_channels}, kernel_size={self._kernel_size}, stride={self._stride}, "
                f"padding={self._padding}, data_format={self._data_format}")


class Conv1D(_ConvNd):
    _n = 1

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCL"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, 0, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format)


class Conv2D(_ConvNd):
    _n = 2

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, 0, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format)


class Conv3D(_ConvNd):
    _n = 3

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCDHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, 0, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format)


class Conv1DTranspose(_ConvNd):
    _n, _transpose = 1, True

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, groups=1,
                 dilation=1, weight_attr=None, bias_attr=None, data_format="NCL"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, output_padding, dilation, groups,
                         "zeros", weight_attr, bias_attr, data_format)


class Conv2DTranspose(_ConvNd):
    _n, _transpose = 2, True

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, dilation=1,
                 groups=1, weight_attr=None, bias_attr=None, data_format="NCHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, output_padding, dilation, groups,
                         "zeros", weight_attr, bias_attr, data_format)


class Conv3DTranspose(_ConvNd):
    _n, _transpose = 3, True

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, dilation=1,
                 groups=1, weight_attr=None, bias_attr=None, data_format="NCDHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, output_padding, dilation, groups,
                         "zeros", weight_attr, bias_attr, data_format)


# ---------------------------------------------------------------------------- norms
class _BatchNormBase(Layer):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format="NCHW", use_global_stats=None, name=None):
        super().__init__()
        self._num_features, self._momentum, self._epsilon = num_features, momentum, epsilon
        self._data_format = data_format
        self._use_global_stats = use_global_stats
        if weight_attr is False:
            self.weight = None
        else:
            self.weight = self.create_parameter([num_features], attr=weight_attr, default_initializer=I.Constant(1.0))
        if bias_attr is False:
            self.bias = None
        else:
            self.bias = self.create_parameter([num_features], attr=bias_attr, is_bias=True)
        dev = _core.default_device()
        mean = _wrap(torch.zeros(num_features, dtype=torch.float32, device=dev))
        var = _wrap(torch.ones(num_features, dtype=torch.float32, device=dev))
        # the reference creates the running statistics as non-trainable parameters named
        # {name}_mean / {name}_variance, else the layer's next two .w names (batch_norm2d_0.w_1 /
        # .w_2, python/paddle/nn/layer/norm.py:627-646): same names here, kept as buffers
        from ...utils import unique_name
        mean.name = name + "_mean" if name else unique_name.generate(self._full_name + ".w")
        var.name = name + "_variance" if name else unique_name.generate(self._full_name + ".w")
        mean.persistable = var.persistable = True
        self.register_buffer("_mean", mean)
        self.register_buffer("_variance", var)

    def forward(self, input):
        return F.batch_norm(input, self._mean, self._variance, self.weight, self.bias, self.training,
                            self._momentum, self._epsilon, self._data_format, self._use_global_stats)

    def extra_repr(self):
        return f"num_features={self._num_features}, momentum={self._momentum}, epsilon={self._epsilon}"


class BatchNorm1D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format="NCL", use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr, data_format, use_global_stats, name)


class BatchNorm2D(_BatchNormBase):
    pass


class BatchNorm3D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format="NCDHW", use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr, data_format, use_global_stats, name)


class BatchNorm(_BatchNormBase):
    """fluid-style BatchNorm(num_channels, act=...)."""

    def __init__(self, num_channels, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None,
                 bias_attr=None, dtype="float32", data_layout="NCHW", in_place=False, moving_mean_name=None,
                 moving_variance_name=None, do_model_average_for_mean_and_var=True, use_global_stats=False,
                 trainable_statistics=False):
        super().__init__(num_channels, momentum, epsilon, param_attr, bias_attr, data_layout, use_global_stats)
        self._act = act

    def forward(self, input):
        y = super().forward(input)
        if self._act:
            y = getattr(F, self._act)(y)
        return y


class SyncBatchNorm(_BatchNormBase):
    """Cross-rank batch statistics (reference: phi/kernels/gpu/sync_batch_norm_kernel.cu):
    per-rank sum/sumsq are all-reduced over the data-parallel group (RCCL), then normalised."""

    def forward(self, input):
        from ...parallel import collective as C
        if not self.training or not C.is_initialized() or C.get_world_size() == 1:
            return super().forward(input)
        return _sync_bn(self, input)

    @classmethod
    def convert_sync_batchnorm(cls, layer):
        out = layer
        if isinstance(layer, _BatchNormBase) and not isinstance(layer, SyncBatchNorm):
            out = SyncBatchNorm(layer._num_features, layer._momentum, layer._epsilon, data_format=layer._data_format)
            if layer.weight is not None:
                out.weight = layer.weight
            if layer.bias is not None:
                out.bias = layer.bias
            out._mean, out._variance = layer._mean, layer._variance
        for name, sub in list(layer._sub_layers.items()):
            out._sub_layers[name] = cls.convert_sync_batchnorm(sub)
        return out


class _SyncBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, rm, rv, momentum, eps, caxis, group):
        import torch.distributed as dist
        dims = [d for d in range(x.dim()) if d != caxis]
        xf = x.float()
        n_local = xf.numel() // xf.shape[caxis]
        stats = torch.stack([xf.sum(dims), (xf * xf).sum(dims)])
        cnt = torch.tensor([float(n_local)], device=x.device)
        dist.all_reduce(stats, group=group)
        dist.all_reduce(cnt, group=group)
        n = cnt.item()
        mean = stats[0] / n
        var = stats[1] / n - mean * mean
        shape = [1] * x.dim()
        shape[caxis] = -1
        rstd = torch.rsqrt(var + eps)
        xhat = (xf - mean.reshape(shape)) * rstd.reshape(shape)
        y = xhat * (w.float().reshape(shape) if w is not None else 1) + (b.float().reshape(shape) if b is not None else 0)
        with torch.no_grad():
            rm.mul_(momentum).add_(mean * (1 - momentum))
            rv.mul_(momentum).add_(var * n / max(n - 1, 1) * (1 - momentum))
        ctx.save_for_backward(xhat, rstd, w)
        ctx.meta = (dims, shape, n, group, caxis)
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, gy):
        import torch.distributed as dist
        xhat, rstd, w = ctx.saved_tensors
        dims, shape, n, group, caxis = ctx.meta
        g = gy.float()
        sums = torch.stack([g.sum(dims), (g * xhat).sum(dims)])
        gw, gb = sums[1].clone(), sums[0].clone()
        dist.all_reduce(sums, group=group)
        wv = w.float().reshape(shape) if w is not None else 1
        gx = (wv * rstd.reshape(shape) / n) * (n * g - sums[0].reshape(shape) - xhat * sums[1].reshape(shape))
        return (gx.to(gy.dtype), None if w is None else gw.to(w.dtype), None if w is None else gb.to(w.dtype),
                None, None, None, None, None, None)


def _sync_bn(layer, x):
    from ...parallel import collective as C
    caxis = x._t.dim() - 1 if layer._data_format in ("NHWC", "NLC", "NDHWC") else 1
    group = C._resolve_group(None)
    y = _SyncBNFn.apply(x._t, None if layer.weight is None else layer.weight._t, None if layer.bias is None else layer.bias._t,
                        layer._mean._t, layer._variance._t, layer._momentum, layer._epsilon, caxis, group)
    return _wrap(y)


class LayerNorm(Layer):
    def __init__(self, normalized_shape, epsilon=1e-05, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        if isinstance(normalized_shape, int):
            normalized_shape = [normalized_shape]
        self._normalized_shape = list(normalized_shape)
        self._epsilon = epsilon
        n = int(np.prod(normalized_shape))
        self.weight = None if weight_attr is False else self.create_parameter([n], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = None if bias_attr is False else self.create_parameter([n], attr=bias_attr, is_bias=True)

    def forward(self, input):
        return F.layer_norm(input, self._normalized_shape, self.weight, self.bias, self._epsilon)

    def extra_repr(self):
        return f"normalized_shape={self._normalized_shape}, epsilon={self._epsilon}"


class RMSNorm(Layer):
    def __init__(self, hidden_size, epsilon=1e-6, weight_attr=None, name=None):
        super().__init__()
        self._epsilon = epsilon
        self.weight = self.create_parameter([hidden_size], attr=weight_attr, default_initializer=I.Constant(1.0))

    def forward(self, x):
        return F.rms_norm(x, self.weight, self._epsilon)


class GroupNorm(Layer):
    def __init__(self, num_groups, num_channels, epsilon=1e-05, weight_attr=None, bias_attr=None, data_format="NCHW", name=None):
        super().__init__()
        self._num_groups, self._epsilon, self._data_format = num_groups, epsilon, data_format
        self.weight = None if weight_attr is False else self.create_parameter([num_channels], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = None if bias_attr is False else self.create_parameter([num_channels], attr=bias_attr, is_bias=True)

    def forward(self, input):
        return F.group_norm(input, self._num_groups, self._epsilon, self.weight, self.bias, self._data_format)


class _InstanceNormBase(Layer):
    _fmt = "NCHW"

    def __init__(self, num_features, epsilon=1e-05, momentum=0.9, weight_attr=None, bias_attr=None, data_format=None, name=None):
        super().__init__()
        self._epsilon, self._data_format = epsilon, data_format or self._fmt
        if weight_attr is False or bias_attr is False:
            self.scale, self.bias = None, None
        else:
            self.scale = self.create_parameter([num_features], attr=weight_attr, default_initializer=I.Constant(1.0))
            self.bias = self.create_parameter([num_features], attr=bias_attr, is_bias=True)

    def forward(self, input):
        return F.instance_norm(input, weight=self.scale, bias=self.bias, eps=self._epsilon, data_format=self._data_format)


class InstanceNorm1D(_InstanceNormBase):
    _fmt = "NCL"


class InstanceNorm2D(_InstanceNormBase):
    _fmt = "NCHW"


class InstanceNorm3D(_InstanceNormBase):
    _fmt = "NCDHW"


class LocalResponseNorm(Layer):
    def __init__(self, size, alpha=0.0001, beta=0.75, k=1.0, data_format="NCHW", name=None):
        super().__init__()
        self.args = (size, alpha, beta, k, data_format)

    def forward(self, input):
        return F.local_response_norm(input, *self.args)


class SpectralNorm(Layer):
    def __init__(self, weight_shape, dim=0, power_iters=1, eps=1e-12, dtype="float32"):
        super().__init__()
        self._dim, self._power_iters, self._eps = dim, power_iters, eps
        h = weight_shape[dim]
        w = int(np.prod(weight_shape)) // h
        self.weight_u = self.create_parameter([h], default_initializer=I.Normal(0.0, 1.0))
        self.weight_u.stop_gradient = True
        self.weight_v = self.create_parameter([w], default_initializer=I.Normal(0.0, 1.0))
        self.weight_v.stop_gradient = True

    def forward(self, weight):
        W = weight._t
        mat = W.movedim(self._dim, 0).reshape(W.shape[self._dim], -1)
        u, v = self.weight_u._t, self.weight_v._t
        with torch.no_grad():
            for _ in range(self._power_iters):
                v.copy_(torch.nn.functional.normalize(mat.t() @ u, dim=0, eps=self._eps))
                u.copy_(torch.nn.functional.normalize(mat @ v, dim=0, eps=self._eps))
        sigma = torch.dot(u, mat @ v)
        return _wrap(W / sigma)


# ---------------------------------------------------------------------------- pooling
class _Pool(Layer):
    def __init__(self, fn, **kw):
        super().__init__()
        self._fn, self._kw = fn, kw

    def forward(self, x):
        return self._fn(x, **self._kw)

    def extra_repr(self):
        return ", ".join(f"{k}={v}" for k, v in self._kw.items())


class AvgPool1D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, exclusive=True, ceil_mode=False, name=None):
        super().__init__(F.avg_pool1d, kernel_size=kernel_size, stride=stride, padding=padding, exclusive=exclusive, ceil_mode=ceil_mode)


class AvgPool2D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
                 data_format="NCHW", name=None):
        super().__init__(F.avg_pool2d, kernel_size=kernel_size, stride=stride, padding=padding, ceil_mode=ceil_mode,
                         exclusive=exclusive, divisor_override=divisor_override, data_format=data_format)


class AvgPool3D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
                 data_format="NCDHW", name=None):
        super().__init__(F.avg_pool3d, kernel_size=kernel_size, stride=stride, padding=padding, ceil_mode=ceil_mode,
                         exclusive=exclusive, divisor_override=divisor_override, data_format=data_format)


class MaxPool1D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, name=None):
        super().__init__(F.max_pool1d, kernel_size=kernel_size, stride=stride, padding=padding, return_mask=return_mask, ceil_mode=ceil_mode)


class MaxPool2D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NCHW", name=None):
        super().__init__(F.max_pool2d, kernel_size=kernel_size, stride=stride, padding=padding, return_mask=return_mask,
                         ceil_mode=ceil_mode, data_format=data_format)


class MaxPool3D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NCDHW", name=None):
        super().__init__(F.max_pool3d, kernel_size=kernel_size, stride=stride, padding=padding, return_mask=return_mask,
                         ceil_mode=ceil_mode, data_format=data_format)


class AdaptiveAvgPool1D(_Pool):
    def __init__(self, output_size, name=None):
        super().__init__(F.adaptive_avg_pool1d, output_size=output_size)


class AdaptiveAvgPool2D(_Pool):
    def __init__(self, output_size, data_format="NCHW", name=None):
        super().__init__(F.adaptive_avg_pool2d, output_size=output_size, data_format=data_format)


class AdaptiveAvgPool3D(_Pool):
    def __init__(self, output_size, data_format="NCDHW", name=None):
        super().__init__(F.adaptive_avg_pool3d, output_size=output_size, data_format=data_format)


class AdaptiveMaxPool1D(_Pool):
    def __init__(self, output_size, return_mask=False, name=None):
        super().__init__(F.adaptive_max_pool1d, output_size=output_size, return_mask=return_mask)


class AdaptiveMaxPool2D(_Pool):
    def __init__(self, output_size, return_mask=False, name=None):
        super().__init__(F.adaptive_max_pool2d, output_size=output_size, return_mask=return_mask)


class AdaptiveMaxPool3D(_Pool):
    def __init__(self, output_size, return_mask=False, name=None):
        super().__init__(F.adaptive_max_pool3d, output_size=output_size, return_mask=return_mask)


class MaxUnPool1D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, data_format="NCL", output_size=None, name=None):
        super().__init__(F.max_unpool1d, kernel_size=kernel_size, stride=stride, padding=padding, data_format=data_format, output_size=output_size)

    def forward(self, x, indices):
        return self._fn(x, indices, **self._kw)


class MaxUnPool2D(MaxUnPool1D):
    def __init__(self, kernel_size, stride=None, padding=0, data_format="NCHW", output_size=None, name=None):
        _Pool.__init__(self, F.max_unpool2d, kernel_size=kernel_size, stride=stride, padding=padding, data_format=data_format, output_size=output_size)


class MaxUnPool3D(MaxUnPool1D):
    def __init__(self, kernel_size, stride=None, padding=0, data_format="NCDHW", output_size=None, name=None):
        _Pool.__init__(self, F.max_unpool3d, kernel_size=kernel_size, stride=stride, padding=padding, data_format=data_format, output_size=output_size)
