"""Common functional ops (reference: python/paddle/nn/functional/{common,input,extension,vision}.py)."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _wrap, convert_dtype
from ...framework.dispatch import register_ops
from ...tensor._helpers import _int_list
from ... import ops as _ops
from ...ops import conv_gemm as _cg

_w = _wrap

__all__ = ["linear", "dropout", "dropout2d", "dropout3d", "alpha_dropout", "pad", "zeropad2d",
           "interpolate", "upsample", "bilinear", "cosine_similarity", "unfold", "fold", "label_smooth",
           "embedding", "one_hot", "class_center_sample", "diag_embed", "sequence_mask", "gather_tree",
           "temporal_shift", "pixel_shuffle", "pixel_unshuffle", "channel_shuffle", "affine_grid",
           "grid_sample", "normalize", "fused_matmul_bias", "linear_bias_gelu"]


def _t(x):
    return x._t if isinstance(x, Tensor) else x


class _LinearBias(torch.autograd.Function):
    """x @ W + b on the own GEMM layouts (ops/gemm.py: NN forward, NT dX, TN dW) with the bias
    gradient from the HIP column-sum kernel; products the own kernels cannot take are counted
    library calls there"""

    @staticmethod
    def forward(ctx, x2d, w, b):
        from ...ops import gemm as _gemm
        ctx.save_for_backward(x2d, w)
        out = _gemm.mm_nn(x2d.contiguous(), w)
        return out.add_(b)

    @staticmethod
    def backward(ctx, gy):
        from ...ops import gemm as _gemm
        from ...ops.conv_gemm import weight_grad
        x2d, w = ctx.saved_tensors
        gy = gy.contiguous()
        dx = _gemm.mm_nt(gy, w) if ctx.needs_input_grad[0] else None
        if ctx.needs_input_grad[1] and ctx.needs_input_grad[2]:
            dw, db = _gemm.mm_tn_db(x2d.contiguous(), gy)   # bias gradient from the dW GEMM's B fragments
        else:
            dw = weight_grad(x2d.contiguous(), gy) if ctx.needs_input_grad[1] else None
            db = _ops.hip.col_sum(gy) if ctx.needs_input_grad[2] else None
        return dx, dw, db


def linear(x, weight, bias=None, name=None):
    """y = x @ W + b with Paddle's [in, out] weight layout (hipBLASLt GEMM + fused bias epilogue;
    PHA_MATMUL_IMPL=hip: the 8-phase MFMA GEMM of gemm8p.hip for forward and both gradients)."""
    xt, wt = x._t, weight._t
    if _cg.linear_ok(xt, wt):
        return _w(_cg.linear(xt, wt, None if bias is None else bias._t))
    if bias is not None and xt.dim() >= 2:
        b = bias._t
        x2d = xt.reshape(-1, xt.shape[-1])
        if _cg.nt_forward_ok(xt, wt) and _ops.fused._use_hip(xt) and b.dtype == xt.dtype:
            out = _cg.LinearNT.apply(x2d, wt, b)
        elif _ops.fused._use_hip(xt) and xt.dtype in (torch.bfloat16, torch.float16) and b.dtype == xt.dtype \
                and wt.dtype == xt.dtype and wt.shape[-1] % 8 == 0:
            out = _LinearBias.apply(x2d, wt, b)
        elif xt.is_cuda:   # fp32 / mixed products: ops/gemm.py (three-term bf16 split for fp32)
            from ...ops import gemm as _gemm
            out = _gemm.matmul(x2d, wt) + b
        else:
            out = torch.addmm(b, x2d, wt)
        return _w(out.reshape(list(xt.shape[:-1]) + [wt.shape[-1]]))
    if bias is None and xt.dim() >= 2 and _cg.nt_forward_ok(xt, wt):
        return _w(_cg.linear_nt(xt, wt))   # the NT product on the cached W^T, like the biased path
    if xt.is_cuda:
        from ...ops import gemm as _gemm
        out = _gemm.matmul(xt, wt)
    else:
        out = torch.matmul(xt, wt)
    if bias is not None:
        out = out + bias._t
    return _w(out)


def fused_matmul_bias(x, y, bias=None, transpose_x=False, transpose_y=False, name=None):
    a, b = _t(x), _t(y)
    if transpose_x:
        a = a.transpose(-1, -2)
    if transpose_y:
        b = b.transpose(-1, -2)
    out = torch.matmul(a, b)
    if bias is not None:
        out = out + _t(bias)
    return _w(out)


def linear_bias_gelu(x, weight, bias, approximate=False):
    """gelu(x @ W + b): GEMM on hipBLASLt, bias+GELU fused in one HIP pass."""
    xt = x._t
    from ...ops import conv_gemm as _cg
    h = _cg.linear(xt, weight._t) if _cg.linear_ok(xt, weight._t) else torch.matmul(xt, weight._t)
    return _w(_ops.bias_gelu(h, bias._t, approximate))


def dropout(x, p=0.5, axis=None, training=True, mode="upscale_in_train", name=None):
    t = _t(x)
    if isinstance(p, Tensor):
        p = float(p._t.item())
    if not training or p == 0.0:
        if mode == "downscale_in_infer" and not training:
            return _w(t * (1.0 - p))
        return _w(t)
    if p == 1.0:
        return _w(torch.zeros_like(t))
    if axis is not None:
        axes = _int_list(axis)
        shape = [t.shape[i] if i in [a % t.dim() for a in axes] else 1 for i in range(t.dim())]
        mask = torch.empty(shape, device=t.device, dtype=t.dtype).bernoulli_(1 - p)
        if mode == "upscale_in_train":
            return _w(t * mask / (1 - p))
        return _w(t * mask)
    if mode == "upscale_in_train":
        return _w(TF.dropout(t, p, True))
    mask = torch.empty_like(t).bernoulli_(1 - p)
    return _w(t * mask)


def dropout2d(x, p=0.5, training=True, data_format="NCHW", name=None):
    t = _t(x)
    if data_format == "NHWC":
        return _w(TF.dropout2d(t.permute(0, 3, 1, 2), p, training).permute(0, 2, 3, 1))
    return _w(TF.dropout2d(t, p, training))


def dropout3d(x, p=0.5, training=True, data_format="NCDHW", name=None):
    t = _t(x)
    if data_format == "NDHWC":
        return _w(TF.dropout3d(t.permute(0, 4, 1, 2, 3), p, training).permute(0, 2, 3, 4, 1))
    return _w(TF.dropout3d(t, p, training))


def alpha_dropout(x, p=0.5, training=True, name=None):
    return _w(TF.alpha_dropout(_t(x), p, training))


def pad(x, pad, mode="constant", value=0.0, data_format="NCHW", name=None):
    t = _t(x)
    pads = _int_list(pad)
    nd = t.dim()
    if len(pads) == 2 * nd:
        # paddle full-rank pad: [d0_before, d0_after, d1_before, ...]
        tp = []
        for i in reversed(range(nd)):
            tp += [pads[2 * i], pads[2 * i + 1]]
        return _w(TF.pad(t, tp, mode=mode, value=value) if mode == "constant" else TF.pad(t, tp, mode=mode))
    channels_last = data_format in ("NHWC", "NLC", "NDHWC")
    if channels_last:
        t = t.movedim(-1, 1)
    # paddle spatial pad order: [left, right, top, bottom, front, back] (last spatial dim first) — same as torch
    if mode == "constant":
        out = TF.pad(t, pads, mode="constant", value=value)
    else:
        out = TF.pad(t, pads, mode={"reflect": "reflect", "replicate": "replicate", "circular": "circular"}[mode])
    if channels_last:
        out = out.movedim(1, -1)
    return _w(out)


def zeropad2d(x, padding, data_format="NCHW", name=None):
    return pad(x, padding, "constant", 0.0, data_format)


def interpolate(x, size=None, scale_factor=None, mode="nearest", align_corners=False, align_mode=0,
                data_format="NCHW", name=None):
    t = _t(x)
    channels_last = data_format in ("NHWC", "NLC", "NDHWC")
    if channels_last:
        t = t.movedim(-1, 1)
    if size is not None:
        size = _int_list(size)
    if isinstance(scale_factor, Tensor):
        scale_factor = scale_factor._t.tolist()
    m = mode.lower()
    linear = m in ("linear", "bilinear", "trilinear")
    if (m == "nearest" and align_corners) or (linear and align_mode == 1 and not align_corners):
        # conventions torch's interpolate has no switch for (reference interp kernels /
        # test_{nearest,bilinear}_interp_v2_op.py oracles): nearest with align_corners rounds
        # ratio * i; align_mode=1 samples at ratio * i (no half-pixel shift)
        out = _interp_indexed(t, size, scale_factor, m == "nearest", align_corners)
    else:
        kw = {}
        if m in ("linear", "bilinear", "bicubic", "trilinear"):
            kw["align_corners"] = align_corners
        out = TF.interpolate(t, size=size, scale_factor=scale_factor, mode=m, **kw)
    if channels_last:
        out = out.movedim(1, -1)
    return _w(out)


upsample = interpolate


def _interp_indexed(t, size, scale_factor, nearest, align_corners):
    """separable nearest / linear resampling of the spatial dims of NC... ``t`` with the
    reference's source coordinates: ratio = (in-1)/(out-1) with align_corners, else 1/scale or
    in/out; nearest: round(ratio*i) (align_corners) / floor(ratio*i); linear: src = ratio*i"""
    sp = t.dim() - 2
    ins = list(t.shape[2:])
    if size is not None:
        outs = list(size) if len(size) == sp else [size[0]] * sp
        scales = [0.0] * sp
    else:
        sf = scale_factor if isinstance(scale_factor, (list, tuple)) else [scale_factor] * sp
        scales = [float(v) for v in sf]
        outs = [int(i * v) for i, v in zip(ins, scales)]
    out = t
    for d in range(sp):
        n_in, n_out, dim = ins[d], outs[d], 2 + d
        if n_out > 1:
            ratio = (n_in - 1.0) / (n_out - 1.0) if align_corners else \
                (1.0 / scales[d] if scales[d] > 0 else n_in / n_out)
        else:
            ratio = 0.0
        i = torch.arange(n_out, dtype=torch.float64, device=t.device)
        src = ratio * i
        if nearest:
            idx = (src + 0.5 if align_corners else src).floor().long().clamp(0, n_in - 1)
            out = out.index_select(dim, idx)
            continue
        i0 = src.floor().long().clamp(0, n_in - 1)
        i1 = (i0 + 1).clamp(max=n_in - 1)
        lam = (src - i0.double()).to(out.dtype)
        shape = [1] * out.dim()
        shape[dim] = n_out
        lam = lam.reshape(shape)
        out = out.index_select(dim, i0) * (1 - lam) + out.index_select(dim, i1) * lam
    return out


def bilinear(x1, x2, weight, bias=None, name=None):
    out = TF.bilinear(_t(x1), _t(x2), _t(weight), None if bias is None else _t(bias).reshape(-1))
    return _w(out)


def cosine_similarity(x1, x2, axis=1, eps=1e-8):
    return _w(TF.cosine_similarity(_t(x1), _t(x2), axis, eps))


def unfold(x, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    p = paddings
    if isinstance(p, (list, tuple)) and len(p) == 4:
        t = TF.pad(_t(x), [p[1], p[3], p[0], p[2]])
        p = 0
    else:
        t = _t(x)
    return _w(TF.unfold(t, kernel_sizes, dilations, p, strides))


def fold(x, output_sizes, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    return _w(TF.fold(_t(x), output_sizes, kernel_sizes, dilations, paddings, strides))


def label_smooth(label, prior_dist=None, epsilon=0.1, name=None):
    t = _t(label)
    k = t.shape[-1]
    if prior_dist is not None:
        return _w((1 - epsilon) * t + epsilon * _t(prior_dist))
    return _w((1 - epsilon) * t + epsilon / k)


def embedding(x, weight, padding_idx=None, sparse=False, name=None):
    w = weight._t
    if padding_idx is not None and padding_idx < 0:
        padding_idx += w.shape[0]
    ids = _t(x)
    out = _ops.embedding(ids, w, padding_idx, sparse)
    if padding_idx is not None:
        # reference lookup_table_v2: rows of padding_idx read as zeros (and get no gradient)
        out = out.masked_fill((ids == padding_idx).unsqueeze(-1), 0)
    return _w(out)


def one_hot(x, num_classes, name=None):
    return _w(TF.one_hot(_t(x).long(), num_classes).float())


def class_center_sample(label, num_classes, num_samples, group=None):
    lab = _t(label)
    pos = torch.unique(lab)
    if pos.numel() < num_samples:
        neg_mask = torch.ones(num_classes, dtype=torch.bool, device=lab.device)
        neg_mask[pos] = False
        neg = torch.nonzero(neg_mask).reshape(-1)
        neg = neg[torch.randperm(neg.numel(), device=lab.device)[: num_samples - pos.numel()]]
        sampled = torch.sort(torch.cat([pos, neg])).values
    else:
        sampled = pos
    remap = torch.full((num_classes,), -1, dtype=torch.int64, device=lab.device)
    remap[sampled] = torch.arange(sampled.numel(), device=lab.device)
    return _w(remap[lab]), _w(sampled)


def diag_embed(input, offset=0, dim1=-2, dim2=-1):
    return _w(torch.diag_embed(_t(input), offset, dim1, dim2))


def sequence_mask(x, maxlen=None, dtype="int64", name=None):
    t = _t(x)
    if maxlen is None:
        maxlen = int(t.max().item())
    elif isinstance(maxlen, Tensor):
        maxlen = int(maxlen._t.item())
    r = torch.arange(maxlen, device=t.device)
    return _w((r < t.unsqueeze(-1)).to(convert_dtype(dtype)))


def gather_tree(ids, parents):
    i, p = _t(ids), _t(parents)
    T = i.shape[0]
    out = torch.empty_like(i)
    out[T - 1] = i[T - 1]
    par = p[T - 1]
    for t in range(T - 2, -1, -1):
        out[t] = torch.gather(i[t], 1, par)
        par = torch.gather(p[t], 1, par)
    return _w(out)


def temporal_shift(x, seg_num, shift_ratio=0.25, name=None, data_format="NCHW"):
    t = _t(x)
    if data_format == "NHWC":
        t = t.permute(0, 3, 1, 2)
    nt, c, h, w = t.shape
    n = nt // seg_num
    t5 = t.reshape(n, seg_num, c, h, w)
    # reference temporal_shift_op: channels [0, c1) take frame t-1, [c1, c2) frame t+1, the rest stay
    c1, c2 = int(c * shift_ratio), int(c * 2 * shift_ratio)
    out = torch.zeros_like(t5)
    out[:, 1:, :c1] = t5[:, :-1, :c1]
    out[:, :-1, c1:c2] = t5[:, 1:, c1:c2]
    out[:, :, c2:] = t5[:, :, c2:]
    out = out.reshape(nt, c, h, w)
    if data_format == "NHWC":
        out = out.permute(0, 2, 3, 1)
    return _w(out)


def pixel_shuffle(x, upscale_factor, data_format="NCHW", name=None):
    t = _t(x)
    if data_format == "NHWC":
        return _w(TF.pixel_shuffle(t.permute(0, 3, 1, 2), upscale_factor).permute(0, 2, 3, 1))
    return _w(TF.pixel_shuffle(t, upscale_factor))


def pixel_unshuffle(x, downscale_factor, data_format="NCHW", name=None):
    t = _t(x)
    if data_format == "NHWC":
        return _w(TF.pixel_unshuffle(t.permute(0, 3, 1, 2), downscale_factor).permute(0, 2, 3, 1))
    return _w(TF.pixel_unshuffle(t, downscale_factor))


def channel_shuffle(x, groups, data_format="NCHW", name=None):
    t = _t(x)
    if data_format == "NHWC":
        n, h, w, c = t.shape
        return _w(t.reshape(n, h, w, groups, c // groups).transpose(3, 4).reshape(n, h, w, c))
    return _w(TF.channel_shuffle(t, groups))


def affine_grid(theta, out_shape, align_corners=True, name=None):
    return _w(TF.affine_grid(_t(theta), _int_list(out_shape), align_corners=align_corners))


def grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=True, name=None):
    return _w(TF.grid_sample(_t(x), _t(grid), mode=mode, padding_mode=padding_mode, align_corners=align_corners))


def normalize(x, p=2, axis=1, epsilon=1e-12, name=None):
    return _w(TF.normalize(_t(x), p, axis, epsilon))


register_ops(globals(), __all__)
