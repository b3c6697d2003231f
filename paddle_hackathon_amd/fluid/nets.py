"""``paddle.fluid.nets`` composite networks (reference: python/paddle/fluid/nets.py)."""
from __future__ import annotations

import math

from . import layers

__all__ = ["simple_img_conv_pool", "sequence_conv_pool", "glu", "scaled_dot_product_attention", "img_conv_group"]


def simple_img_conv_pool(input, num_filters, filter_size, pool_size, pool_stride, pool_padding=0, pool_type="max",
                         global_pooling=False, conv_stride=1, conv_padding=0, conv_dilation=1, conv_groups=1,
                         param_attr=None, bias_attr=None, act=None, use_cudnn=True):
    conv = layers.conv2d(input, num_filters, filter_size, conv_stride, conv_padding, conv_dilation, conv_groups,
                         param_attr, bias_attr, use_cudnn, act)
    return layers.pool2d(conv, pool_size, pool_type, pool_stride, pool_padding, global_pooling, use_cudnn)


def img_conv_group(input, conv_num_filter, pool_size, conv_padding=1, conv_filter_size=3, conv_act=None,
                   param_attr=None, conv_with_batchnorm=False, conv_batchnorm_drop_rate=0.0, pool_stride=1,
                   pool_type="max", use_cudnn=True):
    n = len(conv_num_filter)

    def per(v):
        return list(v) if isinstance(v, (list, tuple)) else [v] * n
    pad, fs, pa, bn, drop = per(conv_padding), per(conv_filter_size), per(param_attr), per(conv_with_batchnorm), \
        per(conv_batchnorm_drop_rate)
    tmp = input
    for i in range(n):
        act = None if bn[i] else conv_act
        tmp = layers.conv2d(tmp, conv_num_filter[i], fs[i], padding=pad[i], param_attr=pa[i], act=act,
                            use_cudnn=use_cudnn)
        if bn[i]:
            tmp = layers.batch_norm(tmp, act=conv_act)
            if abs(drop[i]) > 1e-5:
                tmp = layers.dropout(tmp, drop[i])
    return layers.pool2d(tmp, pool_size, pool_type, pool_stride, use_cudnn=use_cudnn)


def sequence_conv_pool(input, num_filters, filter_size, param_attr=None, act="sigmoid", pool_type="max",
                       bias_attr=None):
    conv = layers.sequence_conv(input, num_filters, filter_size, param_attr=param_attr, bias_attr=bias_attr, act=act)
    return layers.sequence_pool(conv, pool_type)


def glu(input, dim=-1):
    a, b = layers.split(input, 2, dim)
    return layers.elementwise_mul(a, layers.sigmoid(b))


def scaled_dot_product_attention(queries, keys, values, num_heads=1, dropout_rate=0.0):
    """multi-head attention of [B, Lq, D] queries over [B, Lk, D] keys / values (no projections,
    like the reference: heads split the feature dimension)"""
    from .layers._common import T, W
    import torch
    q, k, v = T(queries), T(keys), T(values)
    B, Lq, D = q.shape
    h = num_heads

    def split(x):
        return x.reshape(x.shape[0], x.shape[1], h, -1).transpose(1, 2)
    qh, kh, vh = split(q), split(k), split(v)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(kh.shape[-1])
    w = torch.softmax(s, -1)
    if dropout_rate:
        w = torch.nn.functional.dropout(w, dropout_rate)
    o = (w @ vh).transpose(1, 2).reshape(B, Lq, -1)
    return W(o)
