"""``paddle.incubate.operators.ResNetUnit`` / ``resnet_unit`` (reference:
python/paddle/incubate/operators/resnet_unit.py:39 (resnet_unit), :125 (ResNetUnit);
paddle/fluid/operators/fused/resnet_unit_op.cc / .cu):

    Y = act( BN_x(conv_x(X)) + { BN_z(conv_z(Z))  has_shortcut
                                { Z                fuse_add
                                { 0                otherwise )

with batch statistics in training (running mean / variance updated with ``momentum``) and the
running statistics when ``is_test`` / ``use_global_stats``.

On MI355X the unit is three kernels, not one cuDNN v8 graph: the implicit-GEMM convolution on
the 256-tile MFMA kernels (csrc/kernels/gemm256.hip) with the BN's per-channel sums / sums of
squares reduced in its epilogue (the statistics pass over the conv output is skipped), the
shortcut branch likewise, and one batch_norm.hip pass that normalises, adds the shortcut (or Z)
and applies the ReLU (the fused_bn_add_activation kernel). In backward the BN-add-ReLU gradient
is one pass and the convolutions' dgrad / wgrad run on the same MFMA kernels. NHWC is the native
layout (the filters are [Cout, KH, KW, Cin], exactly the kernels' B operand); NCHW is accepted.
"""
from __future__ import annotations

import numpy as np

from ...framework.core import Tensor, _wrap
from ...framework.dispatch import register_ops

__all__ = ["resnet_unit", "ResNetUnit"]


def _vec(p):
    """a [1, 1, 1, C] / [1, C, 1, 1] BN parameter as a [C] view sharing its storage (the running
    statistics are updated in place through it)"""
    if p is None:
        return None
    t = p._t if isinstance(p, Tensor) else p
    return _wrap(t.view(-1))


def _conv(x, filt, stride, padding, dilation, groups, data_format, filter_layout=None):
    from ...nn import functional as F
    if (filter_layout or ("OHWI" if data_format == "NHWC" else "OIHW")) == "OHWI":
        # [Cout, KH, KW, Cin] -> the OIHW view conv2d takes (autograd flows back)
        filt = _wrap(filt._t.permute(0, 3, 1, 2))
    return F.conv2d(x, filt, None, stride, padding, dilation, groups, data_format)


def resnet_unit(x, filter_x, scale_x, bias_x, mean_x, var_x, z, filter_z, scale_z, bias_z, mean_z, var_z, stride,
                stride_z, padding, dilation, groups, momentum, eps, data_format, fuse_add, has_shortcut,
                use_global_stats, is_test, act, filter_layout=None):
    """functional form with the reference's argument list (resnet_unit_op.cc inputs / attrs).
    ``filter_layout`` (not in the reference): "OHWI" / "OIHW" filters regardless of data_format
    (the fuse pass hands over conv2d's OIHW weights); default: OHWI for NHWC as the reference"""
    from ...nn.functional.norm import batch_norm_act, batch_norm
    if act not in (None, "relu", "identity", ""):
        raise ValueError(f"resnet_unit: act_type {act!r} (relu or none)")
    act = "relu" if act == "relu" else None
    training = not is_test
    conv_x = _conv(x, filter_x, stride, padding, dilation, groups, data_format, filter_layout)
    res = None
    if has_shortcut:
        if z is None or filter_z is None:
            raise ValueError("resnet_unit: has_shortcut needs z and filter_z")
        conv_z = _conv(z, filter_z, stride_z, padding, dilation, groups, data_format, filter_layout)
        res = batch_norm(conv_z, _vec(mean_z), _vec(var_z), _vec(scale_z), _vec(bias_z), training, momentum, eps,
                         data_format, use_global_stats)
    elif fuse_add:
        if z is None:
            raise ValueError("resnet_unit: fuse_add needs z")
        res = z
    return batch_norm_act(conv_x, _vec(mean_x), _vec(var_x), _vec(scale_x), _vec(bias_x), training, momentum, eps,
                          data_format, use_global_stats, residual=res, act=act)


def _layer_base():
    from ...nn.layer.layers import Layer
    return Layer


class ResNetUnit(_layer_base()):
    """conv + BN (+ shortcut conv + BN | + Z) + ReLU as one layer; parameters as the reference's
    (filter_x / scale_x / bias_x / mean_x / var_x and the _z set when ``has_shortcut``)"""

    def __init__(self, num_channels_x, num_filters, filter_size, stride=1, momentum=0.9, eps=1e-5,
                 data_format="NHWC", act="relu", fuse_add=False, has_shortcut=False, use_global_stats=False,
                 is_test=False, filter_x_attr=None, scale_x_attr=None, bias_x_attr=None, moving_mean_x_name=None,
                 moving_var_x_name=None, num_channels_z=1, stride_z=1, filter_z_attr=None, scale_z_attr=None,
                 bias_z_attr=None, moving_mean_z_name=None, moving_var_z_name=None):
        super().__init__()
        from ...nn import initializer as I
        from ...framework.param_attr import ParamAttr
        if data_format not in ("NHWC", "NCHW"):
            raise ValueError(f"conv_format must be one of {{'NHWC', 'NCHW'}}, but got conv_format='{data_format}'")
        self._stride, self._stride_z = stride, stride_z
        self._dilation, self._groups = 1, 1
        self._kernel_size = [filter_size, filter_size]
        self._padding = (filter_size - 1) // 2
        self._momentum, self._eps = momentum, eps
        self._data_format, self._act = data_format, act
        self._fuse_add, self._has_shortcut = fuse_add, has_shortcut
        self._use_global_stats, self._is_test = use_global_stats, is_test
        nchw = data_format == "NCHW"
        bn_shape = [1, num_filters, 1, 1] if nchw else [1, 1, 1, num_filters]

        def fshape(cin):
            return [num_filters, cin, filter_size, filter_size] if nchw else [num_filters, filter_size, filter_size, cin]

        def finit(cin):   # He-normal over the filter's fan-in (the reference's default)
            return I.Normal(0.0, (2.0 / (filter_size * filter_size * cin)) ** 0.5)

        def stats(name, value):
            p = self.create_parameter(shape=bn_shape, dtype="float32",
                                      attr=ParamAttr(name=name, initializer=I.Constant(value), trainable=False))
            p.stop_gradient = True
            return p

        self.filter_x = self.create_parameter(shape=fshape(num_channels_x), attr=filter_x_attr,
                                              default_initializer=finit(num_channels_x))
        self.scale_x = self.create_parameter(shape=bn_shape, attr=scale_x_attr, dtype="float32",
                                             default_initializer=I.Constant(1.0))
        self.bias_x = self.create_parameter(shape=bn_shape, attr=bias_x_attr, dtype="float32", is_bias=True)
        self.mean_x = stats(moving_mean_x_name, 0.0)
        self.var_x = stats(moving_var_x_name, 1.0)
        if has_shortcut:
            self.filter_z = self.create_parameter(shape=fshape(num_channels_z), attr=filter_z_attr,
                                                  default_initializer=finit(num_channels_z))
            self.scale_z = self.create_parameter(shape=bn_shape, attr=scale_z_attr, dtype="float32",
                                                 default_initializer=I.Constant(1.0))
            self.bias_z = self.create_parameter(shape=bn_shape, attr=bias_z_attr, dtype="float32", is_bias=True)
            self.mean_z = stats(moving_mean_z_name, 0.0)
            self.var_z = stats(moving_var_z_name, 1.0)
        else:
            self.filter_z = self.scale_z = self.bias_z = self.mean_z = self.var_z = None

    def forward(self, x, z=None):
        if self._fuse_add and z is None:
            raise ValueError("z can not be None")
        return resnet_unit(x, self.filter_x, self.scale_x, self.bias_x, self.mean_x, self.var_x, z, self.filter_z,
                           self.scale_z, self.bias_z, self.mean_z, self.var_z, self._stride, self._stride_z,
                           self._padding, self._dilation, self._groups, self._momentum, self._eps,
                           self._data_format, self._fuse_add, self._has_shortcut, self._use_global_stats,
                           self._is_test or not self.training, self._act)


_ = np
register_ops(globals(), ["resnet_unit"])
