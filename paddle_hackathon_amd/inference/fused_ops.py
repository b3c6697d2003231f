"""Fused ops the inference passes rewrite into (reference: paddle/fluid/operators/fused/
fc_op / conv_fusion_op / skip_layernorm_op / multihead_matmul_op).

Plain functions over our Tensors: the passes place them into Programs as OpDescs (qualified
name = this module), so they serialise into ProgramDescs like any other op. GPU paths are the
fused HIP kernels (bias+GELU, residual-add+LayerNorm, BN-folded conv + residual + ReLU, flash
attention)."""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from ..framework.core import _wrap
from .. import ops as _ops


def _t(x):
    return None if x is None else x._t


def fc(x, weight, bias=None, activation=None):
    """x @ W (+ b) with relu / gelu folded in (W: [in, out] as the reference's fc)"""
    from ..nn.functional.common import linear
    if activation == "gelu" and bias is not None:
        h = linear(x, weight)._t
        return _wrap(_ops.fused.bias_gelu(h, bias._t.to(h.dtype)))
    out = linear(x, weight, bias)._t
    if activation == "relu":
        out = torch.relu(out)
    elif activation == "gelu":
        out = _ops.fused.gelu(out)
    elif activation:
        raise ValueError(f"fc: unsupported activation {activation}")
    return _wrap(out)


def conv2d_fusion(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCHW",
                  residual=None, act=None):
    """conv2d (BN folded into weight / bias) + residual add + ReLU"""
    from ..nn.functional.conv import conv2d
    out = conv2d.__wrapped_op__(x, weight, bias, stride, padding, dilation, groups, data_format) \
        if hasattr(conv2d, "__wrapped_op__") else conv2d(x, weight, bias, stride, padding, dilation, groups, data_format)
    t = out._t
    if residual is not None:
        t = t + residual._t
    if act == "relu":
        t = torch.relu(t)
    elif act is not None:
        raise ValueError(f"conv2d_fusion: unsupported activation {act}")
    return _wrap(t)


def skip_layernorm(x, y, weight=None, bias=None, epsilon=1e-5):
    """LayerNorm(x + y) over the last dim in one pass"""
    xt, yt = x._t, y._t
    H = xt.shape[-1]
    w = weight._t if weight is not None else torch.ones(H, dtype=xt.dtype, device=xt.device)
    _, out = _ops.fused.add_layer_norm(xt.contiguous(), yt.contiguous(), w, _t(bias), float(epsilon))
    return _wrap(out)


def multihead_attention(q, k, v, mask=None, scale=1.0):
    """softmax(q k^T * scale + mask) v for [B, H, S, D] operands on the flash kernels"""
    qt, kt, vt = (t._t.transpose(1, 2) for t in (q, k, v))      # -> [B, S, H, D]
    m = _t(mask)
    o = _ops.fused.flash_attention(qt.contiguous(), kt.contiguous(), vt.contiguous(), causal=False, dropout_p=0.0,
                                   scale=float(scale), training=False, mask=m)
    return _wrap(o.transpose(1, 2))


def scale_inference(x, scale=1.0):
    return _wrap(x._t * scale)


def _reference_attention(q, k, v, mask, scale):   # used by tests only
    s = torch.matmul(q, k.transpose(-1, -2)) * scale
    if mask is not None:
        s = s + mask
    return torch.matmul(TF.softmax(s, -1), v)
