"""Normalisation (reference: python/paddle/nn/functional/norm.py,
phi/kernels/gpu/{batch_norm,layer_norm,group_norm,instance_norm}_kernel.cu).
LayerNorm on HIP tensors runs our gfx950 kernel (ops.layer_norm)."""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _wrap
from ...framework.dispatch import register_ops
from ... import ops as _ops

_w = _wrap

__all__ = ["batch_norm", "layer_norm", "instance_norm", "group_norm", "local_response_norm", "rms_norm"]


def _t(x):
    return None if x is None else (x._t if isinstance(x, Tensor) else x)


def batch_norm(x, running_mean, running_var, weight, bias, training=False, momentum=0.9, epsilon=1e-05,
               data_format="NCHW", use_global_stats=None, name=None):
    t = x._t
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    if cl:
        t = t.movedim(-1, 1)
        if t.dim() == 4:
            t = t.contiguous(memory_format=torch.channels_last) if not t.is_contiguous(memory_format=torch.channels_last) else t
    use_batch = training and not use_global_stats
    rm, rv = _t(running_mean), _t(running_var)
    out = TF.batch_norm(t, rm, rv, _t(weight), _t(bias), use_batch, 1.0 - momentum, epsilon)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


def layer_norm(x, normalized_shape, weight=None, bias=None, epsilon=1e-05, name=None):
    if isinstance(normalized_shape, int):
        normalized_shape = [normalized_shape]
    return _w(_ops.layer_norm(x._t, list(normalized_shape), _t(weight), _t(bias), epsilon))


def rms_norm(x, weight=None, epsilon=1e-6, name=None):
    return _w(_ops.rms_norm(x._t, _t(weight), epsilon))


def instance_norm(x, running_mean=None, running_var=None, weight=None, bias=None, use_input_stats=True,
                  momentum=0.9, eps=1e-05, data_format="NCHW", name=None):
    t = x._t
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    if cl:
        t = t.movedim(-1, 1)
    out = TF.instance_norm(t, _t(running_mean), _t(running_var), _t(weight), _t(bias), use_input_stats, 1 - momentum, eps)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


def group_norm(x, num_groups, epsilon=1e-05, weight=None, bias=None, data_format="NCHW", name=None):
    t = x._t
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    if cl:
        t = t.movedim(-1, 1)
    out = TF.group_norm(t, num_groups, _t(weight), _t(bias), epsilon)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


def local_response_norm(x, size, alpha=1e-4, beta=0.75, k=1.0, data_format="NCHW", name=None):
    t = x._t
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    if cl:
        t = t.movedim(-1, 1)
    out = TF.local_response_norm(t, size, alpha, beta, k)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


register_ops(globals(), __all__)
