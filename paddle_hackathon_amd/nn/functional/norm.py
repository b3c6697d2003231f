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
    """Channels-last inputs (NHWC/NLC/NDHWC, and NCHW tensors whose memory is channels-last — the
    own convolutions' outputs) run the fused HIP BN kernels; other channels-first tensors use the
    library kernel (reference: nn/functional/norm.py:batch_norm)."""
    return batch_norm_act(x, running_mean, running_var, weight, bias, training, momentum, epsilon, data_format,
                          use_global_stats)


def batch_norm_act(x, running_mean, running_var, weight, bias, training=False, momentum=0.9, epsilon=1e-05,
                   data_format="NCHW", use_global_stats=None, residual=None, act=None):
    """BN (+ residual add) (+ ReLU) in one pass — the fused_bn_add_activation op of the reference
    (fluid/operators/fused/fused_bn_add_activation_op.cu), used by the ResNet blocks."""
    if act not in (None, "relu"):
        raise ValueError(f"unsupported fused activation {act}")
    t = x._t
    cl = data_format in ("NHWC", "NLC", "NDHWC") or (t.dim() == 2)
    use_batch = training and not use_global_stats
    rm, rv = _t(running_mean), _t(running_var)
    res = _t(residual)
    back = False
    if not cl and t.is_cuda and t.dim() == 4:
        # NCHW tensor in channels-last memory (what the own convolutions return): the NHWC kernels
        # on the NHWC view, the result viewed back as NCHW
        from .conv import nhwc_view
        v = nhwc_view(t)
        if v is not None:
            t, cl, back = v, True, True
            if res is not None:
                res = res.permute(0, 2, 3, 1)
    if cl:
        if res is not None:
            res = res.contiguous()
        if use_batch:
            out = _ops.fused.batch_norm_train(t.contiguous(), _t(weight), _t(bias), rm, rv, momentum, epsilon, -1,
                                              residual=res, relu=act == "relu")
        else:
            out = _ops.fused.batch_norm_infer(t.contiguous(), _t(weight), _t(bias), rm, rv, epsilon, -1, residual=res,
                                              relu=act == "relu")
        return _w(out.permute(0, 3, 1, 2) if back else out)
    out = TF.batch_norm(t, rm, rv, _t(weight), _t(bias), use_batch, 1.0 - momentum, epsilon)
    if res is not None:
        out = out + res
    if act == "relu":
        out = torch.relu(out)
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
