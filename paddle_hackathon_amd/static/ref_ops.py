"""Converters for reference-written ProgramDesc ops beyond the core inference set of
static/serialize.py: activations, comparisons / logic, shape and indexing ops, interpolation,
normalisation, detection heads and the 1.x control-flow ops (conditional_block / select_input /
while / tensor arrays) that the reference's exported inference models contain. Slot and attribute
names follow paddle/fluid/operators/*_op.cc (and the phi op yaml of the 2.x ops).

A converter is ``conv(reader, ins, attrs) -> (fn, kwargs, out)`` with ``out`` one output slot name,
a tuple of slot names (one Variable each), or ``("list", slot)`` (all Variables of the slot);
control-flow converters build their OpDesc themselves (``_CF``). Every implementation is a
module-level function, so a loaded program serialises again by qualified name.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as TF

from ..framework import core as _core
from ..framework.core import Tensor, _wrap
from . import proto as pb


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def _one(r, ins, slot):
    return r.var(ins[slot][0]) if ins.get(slot) else None


def _many(r, ins, slot):
    return [r.var(n) for n in ins.get(slot, [])]


def _dt(code, default=torch.float32):
    return pb.dtype_of(code) if code is not None and code >= 0 else default


# ----------------------------------------------------------------------------- implementations
def unary_op(x, op, **kw):
    t = _t(x)
    f = {
        "abs": torch.abs, "acos": torch.acos, "asin": torch.asin, "atan": torch.atan, "ceil": torch.ceil,
        "cos": torch.cos, "cosh": torch.cosh, "floor": torch.floor, "log": torch.log, "log1p": torch.log1p,
        "log2": torch.log2, "log10": torch.log10, "reciprocal": torch.reciprocal, "round": torch.round,
        "rsqrt": torch.rsqrt, "sin": torch.sin, "sinh": torch.sinh, "square": torch.square, "tan": torch.tan,
        "softsign": TF.softsign, "expm1": torch.expm1, "erf": torch.erf, "sign": torch.sign,
        "logsigmoid": TF.logsigmoid, "tanh_shrink": lambda v: v - torch.tanh(v), "logical_not": torch.logical_not,
        "isfinite_v2": torch.isfinite, "isnan_v2": torch.isnan, "isinf_v2": torch.isinf,
        "relu6": lambda v: v.clamp(0, kw.get("threshold", 6.0)),
        "leaky_relu": lambda v: TF.leaky_relu(v, kw.get("alpha", 0.02)),
        "elu": lambda v: TF.elu(v, kw.get("alpha", 1.0)),
        "selu": lambda v: kw.get("scale", 1.0507009873554805) * torch.where(
            v > 0, v, kw.get("alpha", 1.6732632423543772) * (torch.exp(v) - 1)),
        "swish": lambda v: v * torch.sigmoid(kw.get("beta", 1.0) * v),
        "hard_swish": lambda v: v * (v + kw.get("offset", 3.0)).clamp(0, kw.get("threshold", 6.0)) / kw.get("scale", 6.0),
        "hard_sigmoid": lambda v: (kw.get("slope", 0.2) * v + kw.get("offset", 0.5)).clamp(0, 1),
        "softshrink": lambda v: TF.softshrink(v, kw.get("lambda", 0.5)),
        "hard_shrink": lambda v: TF.hardshrink(v, kw.get("threshold", 0.5)),
        "thresholded_relu": lambda v: torch.where(v > kw.get("threshold", 1.0), v, torch.zeros_like(v)),
        "brelu": lambda v: v.clamp(kw.get("t_min", 0.0), kw.get("t_max", 24.0)),
        "stanh": lambda v: kw.get("scale_b", 1.7159) * torch.tanh(kw.get("scale_a", 0.67) * v),
        "soft_relu": lambda v: torch.log1p(torch.exp(v.clamp(-kw.get("threshold", 40.0), kw.get("threshold", 40.0)))),
        "softplus": lambda v: TF.softplus(v, kw.get("beta", 1.0), kw.get("threshold", 20.0)),
        "mish": lambda v: v * torch.tanh(TF.softplus(v)),
        "log_softmax": lambda v: torch.log_softmax(v, kw.get("axis", -1)),
        "squared_l2_norm": lambda v: (v * v).sum().reshape(1),
        "mean": lambda v: v.mean().reshape(1),
        "fill_zeros_like": torch.zeros_like,
        "assign": lambda v: v.clone(),
    }[op]
    return _wrap(f(t))


def binary_op(x, y, op, axis=-1):
    a, b = _t(x), _t(y)
    if axis not in (-1, None) and b.dim() < a.dim():
        b = b.reshape([1] * axis + list(b.shape) + [1] * (a.dim() - axis - b.dim()))
    f = {"elementwise_mod": torch.remainder, "elementwise_floordiv": lambda u, v: torch.div(u, v, rounding_mode="floor"),
         "less_than": torch.lt, "less_equal": torch.le, "greater_than": torch.gt, "greater_equal": torch.ge,
         "equal": torch.eq, "not_equal": torch.ne, "logical_and": torch.logical_and,
         "logical_or": torch.logical_or, "logical_xor": torch.logical_xor, "bmm": torch.bmm,
         "dot": lambda u, v: (u * v).sum(-1)}[op]
    return _wrap(f(a, b))


def matmul_v1(x, y, transpose_X=False, transpose_Y=False, alpha=1.0):
    a, b = _t(x), _t(y)
    if transpose_X and a.dim() > 1:
        a = a.transpose(-1, -2)
    if transpose_Y and b.dim() > 1:
        b = b.transpose(-1, -2)
    out = torch.matmul(a, b)
    return _wrap(out * alpha if alpha != 1.0 else out)


def prelu_op(x, alpha, mode="all", data_format="NCHW"):
    t, a = _t(x), _t(alpha)
    if mode == "channel":
        shp = [1] * t.dim()
        shp[1 if data_format == "NCHW" else -1] = -1
        a = a.reshape(shp)
    elif mode == "element":
        a = a.reshape([1] + list(t.shape[1:]))
    return _wrap(torch.where(t > 0, t, a * t))


def stack_op(xs, axis=0):
    return _wrap(torch.stack([_t(x) for x in xs], axis))


def unstack_op(x, axis=0):
    return [_wrap(v) for v in torch.unbind(_t(x), axis)]


def split_op(x, num=0, sections=(), axis=0):
    t = _t(x)
    if num:
        return [_wrap(v) for v in torch.chunk(t, num, axis)]
    secs = list(sections)
    if -1 in secs:
        secs[secs.index(-1)] = t.shape[axis] - (sum(secs) + 1)
    return [_wrap(v) for v in torch.split(t, secs, axis)]


def gather_op(x, index, axis=0):
    return _wrap(torch.index_select(_t(x), axis, _t(index).reshape(-1).long()))


def gather_nd_op(x, index):
    t, idx = _t(x), _t(index).long()
    k = idx.shape[-1]
    flat = idx.reshape(-1, k)
    out = t[tuple(flat[:, i] for i in range(k))]
    return _wrap(out.reshape(list(idx.shape[:-1]) + list(t.shape[k:])))


def shape_op(x):
    return _wrap(torch.tensor(list(_t(x).shape), dtype=torch.int32, device=_core.default_device()))


def size_op(x):
    return _wrap(torch.tensor([_t(x).numel()], dtype=torch.int64, device=_core.default_device()))


def expand_v2_op(x, shape):
    t = _t(x)
    shp = [t.shape[i - (len(shape) - t.dim())] if s == -1 else s for i, s in enumerate(shape)]
    return _wrap(t.expand(shp).contiguous())


def expand_op(x, expand_times):
    return _wrap(_t(x).repeat(*expand_times))


def expand_as_op(x, target_shape):
    t = _t(x)
    return _wrap(t.expand(list(target_shape)).contiguous())


def tile_op(x, repeat_times):
    t = _t(x)
    reps = list(repeat_times)
    if len(reps) < t.dim():
        reps = [1] * (t.dim() - len(reps)) + reps
    return _wrap(t.repeat(*reps))


def flatten2_op(x, axis=1):
    t = _t(x)
    return _wrap(t.reshape(int(np.prod(t.shape[:axis])) if axis else 1, -1))


def reshape_v1(x, shape):
    t = _t(x)
    shp = [t.shape[i] if s == 0 else s for i, s in enumerate(shape)]
    return _wrap(t.reshape(shp))


def transpose_v1(x, axis):
    return _wrap(_t(x).permute(*axis))


def squeeze_v1(x, axes=()):
    t = _t(x)
    axes = [a % t.dim() for a in axes] if axes else [i for i, s in enumerate(t.shape) if s == 1]
    return _wrap(t.reshape([s for i, s in enumerate(t.shape) if not (i in axes and s == 1)]))


def unsqueeze_v1(x, axes):
    t = _t(x)
    for a in axes:
        t = t.unsqueeze(a if a >= 0 else a + t.dim() + 1)
    return _wrap(t)


def arg_op(x, op="arg_max", axis=-1, keepdims=False, flatten=False, dtype=3):
    t = _t(x)
    if flatten:
        t = t.reshape(-1)
        axis = 0
    f = torch.argmax if op == "arg_max" else torch.argmin
    return _wrap(f(t, axis, keepdim=keepdims).to(_dt(dtype, torch.int64)))


def top_k_op(x, k=1, axis=-1, largest=True, sorted=True):
    v, i = torch.topk(_t(x), k, axis, largest, sorted)
    return _wrap(v), _wrap(i)


def argsort_op(x, axis=-1, descending=False):
    v, i = torch.sort(_t(x), dim=axis, descending=descending, stable=True)
    return _wrap(v), _wrap(i)


def cumsum_op(x, axis=-1, exclusive=False, reverse=False, flatten=False):
    t = _t(x)
    if flatten:
        t, axis = t.reshape(-1), 0
    if reverse:
        t = t.flip(axis)
    out = torch.cumsum(t, axis)
    if exclusive:
        out = out - t
    return _wrap(out.flip(axis) if reverse else out)


def clip_op(x, min=-3.4e38, max=3.4e38):
    return _wrap(_t(x).clamp(min, max))


def where_op(condition, x, y):
    return _wrap(torch.where(_t(condition).bool(), _t(x), _t(y)))


def where_index_op(condition):
    return _wrap(torch.nonzero(_t(condition).bool()).long())


def one_hot_op(x, depth, v1=False):
    ids = _t(x).long()
    if v1 and ids.dim() > 1 and ids.shape[-1] == 1:
        ids = ids.squeeze(-1)
    return _wrap(TF.one_hot(ids, depth).float())


def range_op(start, end, step):
    s, e, st = (_t(v).reshape(-1)[0].item() for v in (start, end, step))
    return _wrap(torch.arange(s, e, st, device=_core.default_device()).to(_t(start).dtype))


def linspace_op(start, stop, num, dtype=5):
    s, e, n = (_t(v).reshape(-1)[0].item() for v in (start, stop, num))
    return _wrap(torch.linspace(s, e, int(n), device=_core.default_device()).to(_dt(dtype)))


def fill_any_like_op(x, value=0.0, dtype=-1):
    t = _t(x)
    return _wrap(torch.full_like(t, value, dtype=_dt(dtype, t.dtype)))


def fill_constant_bsl_op(input, shape, value=0.0, dtype=5, input_dim_idx=0, output_dim_idx=0):
    shp = list(shape)
    shp[output_dim_idx] = _t(input).shape[input_dim_idx]
    return _wrap(torch.full(shp, value, dtype=_dt(dtype), device=_core.default_device()))


def assign_value_op(shape, dtype, values):
    return _wrap(torch.tensor(values, dtype=_dt(dtype), device=_core.default_device()).reshape(shape))


def pad_op(x, paddings, pad_value=0.0):
    t = _t(x)
    flat = []
    for i in reversed(range(t.dim())):
        flat += [paddings[2 * i], paddings[2 * i + 1]]
    return _wrap(TF.pad(t, flat, value=pad_value))


def pad_nd_op(x, paddings, mode="constant", value=0.0, data_format="NCHW"):
    """pad2d paddings (top, bottom, left, right); pad3d (left, right, top, bottom, front, back)"""
    t = _t(x)
    cl = data_format in ("NHWC", "NDHWC")
    if cl:
        t = t.movedim(-1, 1)
    p = list(paddings)
    if t.dim() == 4:
        flat = [p[2], p[3], p[0], p[1]] if len(p) == 4 else p
    else:
        flat = p
    m = {"constant": "constant", "reflect": "reflect", "edge": "replicate", "replicate": "replicate",
         "circular": "circular"}[mode]
    y = TF.pad(t, flat, mode=m, value=value) if m == "constant" else TF.pad(t, flat, mode=m)
    return _wrap(y.movedim(1, -1) if cl else y)


def strided_slice_op(x, axes, starts, ends, strides, decrease_axis=()):
    t = _t(x)
    for a, s, e, st in zip(axes, starts, ends, strides):
        # the reference clamps start / end into the dim like Python slicing (negative values count
        # from the end; an end past the front with a negative stride runs through index 0)
        idx = list(range(*slice(s, e, st).indices(t.shape[a])))
        t = t.index_select(a, torch.tensor(idx, dtype=torch.long, device=t.device))
    if decrease_axis:
        t = t.squeeze(tuple(decrease_axis))
    return _wrap(t)


def index_select_op(x, index, dim=0):
    return _wrap(torch.index_select(_t(x), dim, _t(index).long()))


def scatter_op(x, ids, updates, overwrite=True):
    t = _t(x).clone()
    i = _t(ids).reshape(-1).long()
    if overwrite:
        t[i] = _t(updates)
    else:
        t[i] = 0
        t = t.index_add(0, i, _t(updates))
    return _wrap(t)


def tril_triu_op(x, diagonal=0, lower=False):
    t = _t(x)
    return _wrap(torch.tril(t, diagonal) if lower else torch.triu(t, diagonal))


def interp_op(x, out_h=-1, out_w=-1, out_d=-1, scale=(), interp_method="bilinear", align_corners=True,
              align_mode=1, data_layout="NCHW"):
    from ..nn import functional as F
    t = _t(x)
    nd = t.dim() - 2
    size = None
    if (out_h or -1) > 0:
        size = [out_d, out_h, out_w][3 - nd:] if nd != 1 else [out_w]
    sc = list(scale) if scale else None
    if sc and len(sc) == 1:
        sc = sc * nd
    mode = {"bilinear": "bilinear", "nearest": "nearest", "linear": "linear", "bicubic": "bicubic",
            "trilinear": "trilinear"}[interp_method]
    return F.interpolate(_wrap(t), size=size, scale_factor=None if size else sc, mode=mode,
                         align_corners=align_corners if mode != "nearest" else False, align_mode=align_mode,
                         data_format=data_layout)


def pixel_shuffle_op(x, upscale_factor, data_format="NCHW"):
    t = _t(x)
    if data_format == "NHWC":
        return _wrap(TF.pixel_shuffle(t.permute(0, 3, 1, 2), upscale_factor).permute(0, 2, 3, 1))
    return _wrap(TF.pixel_shuffle(t, upscale_factor))


def shuffle_channel_op(x, group):
    t = _t(x)
    B, C, H, W = t.shape
    return _wrap(t.reshape(B, group, C // group, H, W).transpose(1, 2).reshape(B, C, H, W))


def affine_channel_op(x, scale, bias, data_layout="NCHW"):
    t = _t(x)
    shp = [1] * t.dim()
    shp[1 if data_layout == "NCHW" else -1] = -1
    return _wrap(t * _t(scale).reshape(shp) + _t(bias).reshape(shp))


def conv_transpose_op(x, weight, bias=None, strides=(1, 1), paddings=(0, 0), dilations=(1, 1), groups=1,
                      output_size=(), data_format="NCHW", padding_algorithm="EXPLICIT"):
    from ..nn import functional as F
    nd = _t(x).dim() - 2
    f = F.conv2d_transpose if nd == 2 else F.conv3d_transpose
    pad = padding_algorithm if padding_algorithm in ("SAME", "VALID") else list(paddings)
    osz = list(output_size) or None
    if nd == 2:
        return f(x, weight, bias, list(strides), pad, 0, list(dilations), groups, osz, data_format)
    return f(x, weight, bias, list(strides), pad, 0, groups, list(dilations), osz, data_format)


def conv3d_op(x, weight, bias=None, strides=(1, 1, 1), paddings=(0, 0, 0), dilations=(1, 1, 1), groups=1,
              data_format="NCDHW"):
    from ..nn import functional as F
    return F.conv3d(x, weight, bias, list(strides), list(paddings), list(dilations), groups, data_format)


def pool3d_op(x, pooling_type="max", ksize=(1, 1, 1), strides=(1, 1, 1), paddings=(0, 0, 0), global_pooling=False,
              exclusive=True, ceil_mode=False, data_format="NCDHW"):
    t = _t(x)
    if global_pooling:
        return _wrap(t.amax((2, 3, 4), keepdim=True) if pooling_type == "max" else t.mean((2, 3, 4), keepdim=True))
    if pooling_type == "max":
        return _wrap(TF.max_pool3d(t, list(ksize), list(strides), list(paddings), ceil_mode=ceil_mode))
    return _wrap(TF.avg_pool3d(t, list(ksize), list(strides), list(paddings), ceil_mode=ceil_mode,
                               count_include_pad=not exclusive))


def instance_norm_op(x, scale=None, bias=None, epsilon=1e-5):
    t = _t(x)
    return _wrap(TF.instance_norm(t, weight=_t(scale) if scale is not None else None,
                                  bias=_t(bias) if bias is not None else None, eps=epsilon))


def group_norm_op(x, scale=None, bias=None, epsilon=1e-5, groups=1, data_layout="NCHW"):
    t = _t(x)
    cl = data_layout == "NHWC"
    if cl:
        t = t.movedim(-1, 1)
    y = TF.group_norm(t, groups, _t(scale) if scale is not None else None, _t(bias) if bias is not None else None,
                      epsilon)
    return _wrap(y.movedim(1, -1) if cl else y)


def sum_op(xs):
    out = _t(xs[0])
    for v in xs[1:]:
        out = out + _t(v)
    return _wrap(out)


def reduce_op(x, op, dim=(), keep_dim=False, reduce_all=False):
    t = _t(x)
    dims = tuple(range(t.dim())) if reduce_all or not dim else tuple(d % t.dim() for d in dim)
    if op == "reduce_min":
        return _wrap(t.amin(dims, keepdim=keep_dim))
    if op == "reduce_prod":
        out = t
        for d in sorted(dims, reverse=True):
            out = out.prod(d, keepdim=keep_dim)
        return _wrap(out)
    if op == "reduce_all":
        return _wrap(t.bool().all(dims[0], keepdim=keep_dim) if len(dims) == 1 else t.bool().all())
    return _wrap(t.bool().any(dims[0], keepdim=keep_dim) if len(dims) == 1 else t.bool().any())


def p_norm_op(x, porder=2.0, axis=-1, keepdim=False, epsilon=1e-12):
    return _wrap(torch.linalg.vector_norm(_t(x), porder, dim=axis, keepdim=keepdim))


def norm_op(x, axis=1, epsilon=1e-10):
    t = _t(x)
    n = torch.sqrt((t * t).sum(axis, keepdim=True) + epsilon)
    return _wrap(t / n), _wrap(n)


def lookup_v1_op(ids, w, padding_idx=-1):
    i = _t(ids).long()
    if i.dim() > 1 and i.shape[-1] == 1:
        i = i.squeeze(-1)
    return _wrap(TF.embedding(i, _t(w), padding_idx=None if padding_idx == -1 else padding_idx))


def roi_align_op(x, rois, rois_num=None, pooled_height=1, pooled_width=1, spatial_scale=1.0, sampling_ratio=-1,
                 aligned=False):
    from ..vision import ops as V
    num = rois_num if rois_num is not None else _wrap(torch.tensor([_t(rois).shape[0]], dtype=torch.int32))
    return V.roi_align(x, rois, num, (pooled_height, pooled_width), spatial_scale, sampling_ratio, aligned)


def prior_box_op(input, image, min_sizes, max_sizes=(), aspect_ratios=(1.0,), variances=(0.1, 0.1, 0.2, 0.2),
                 flip=False, clip=False, step_w=0.0, step_h=0.0, offset=0.5, min_max_aspect_ratios_order=False):
    from ..vision import ops as V
    return V.prior_box(input, image, list(min_sizes), list(max_sizes) or None, list(aspect_ratios), list(variances),
                       flip, clip, [step_w, step_h], offset, min_max_aspect_ratios_order)


def box_coder_op(prior_box, prior_box_var, target_box, code_type="encode_center_size", box_normalized=True, axis=0,
                 variance=()):
    from ..vision import ops as V
    pv = prior_box_var if prior_box_var is not None else (list(variance) or None)
    return V.box_coder(prior_box, pv, target_box, code_type, box_normalized, axis)


def multiclass_nms_op(bboxes, scores, score_threshold=0.05, nms_top_k=-1, keep_top_k=-1, nms_threshold=0.3,
                      normalized=True, nms_eta=1.0, background_label=0):
    from ..fluid.layers import detection as D
    return D.multiclass_nms(bboxes, scores, score_threshold, nms_top_k, keep_top_k, nms_threshold, normalized,
                            nms_eta, background_label)


def yolo_box_op(x, img_size, anchors, class_num, conf_thresh, downsample_ratio, clip_bbox=True, scale_x_y=1.0):
    from ..vision import ops as V
    return V.yolo_box(x, img_size, list(anchors), class_num, conf_thresh, downsample_ratio, clip_bbox,
                      scale_x_y=scale_x_y)


def random_op(shape, op="uniform_random", min=-1.0, max=1.0, mean=0.0, std=1.0, seed=0, dtype=5):
    g = torch.Generator(device=_core.default_device())
    if seed:
        g.manual_seed(int(seed))
    t = torch.empty(list(shape), dtype=_dt(dtype), device=_core.default_device())
    return _wrap(t.uniform_(min, max, generator=g) if op == "uniform_random" else t.normal_(mean, std, generator=g))


def masked_select_op(x, mask):
    return _wrap(torch.masked_select(_t(x), _t(mask).bool()))


def meshgrid_op(xs):
    return [_wrap(v) for v in torch.meshgrid(*[_t(x) for x in xs], indexing="ij")]


def roll_op(x, shifts, axis=()):
    return _wrap(torch.roll(_t(x), list(shifts), list(axis) or None))


def flip_op(x, axis):
    return _wrap(torch.flip(_t(x), list(axis)))


def grid_sampler_op(x, grid, align_corners=True, mode="bilinear", padding_mode="zeros"):
    return _wrap(TF.grid_sample(_t(x), _t(grid), mode=mode, padding_mode=padding_mode, align_corners=align_corners))


def unfold_op(x, kernel_sizes, strides, paddings, dilations):
    p = list(paddings)
    t = _t(x)
    if len(p) == 4 and (p[0] != p[2] or p[1] != p[3]):
        t = TF.pad(t, [p[1], p[3], p[0], p[2]])
        p = [0, 0]
    return _wrap(TF.unfold(t, list(kernel_sizes), list(dilations), p[:2], list(strides)))


def _fluid(name):
    from ..fluid import layers as L
    f = getattr(L, name)
    return getattr(f, "__wrapped_op__", f)


# ----------------------------------------------------------------------------- converters
def _unary(op, **attr_defaults):
    def conv(r, ins, at):
        kw = {k: at.get(k, v) for k, v in attr_defaults.items()}
        return unary_op, {"x": _one(r, ins, "X"), "op": op, **kw}, "Out"
    return conv


def _binary(op):
    def conv(r, ins, at):
        return binary_op, {"x": _one(r, ins, "X"), "y": _one(r, ins, "Y"), "op": op, "axis": at.get("axis", -1)}, "Out"
    return conv


def _reduce(op):
    def conv(r, ins, at):
        return reduce_op, {"x": _one(r, ins, "X"), "op": op, "dim": at.get("dim", []),
                           "keep_dim": at.get("keep_dim", False), "reduce_all": at.get("reduce_all", False)}, "Out"
    return conv


def _interp(method):
    def conv(r, ins, at):
        return interp_op, {"x": _one(r, ins, "X"), "out_h": at.get("out_h", -1), "out_w": at.get("out_w", -1),
                           "out_d": at.get("out_d", -1), "scale": at.get("scale", []) if isinstance(
                               at.get("scale", []), list) else [at["scale"]] if at.get("scale", 0) > 0 else [],
                           "interp_method": at.get("interp_method", method),
                           "align_corners": at.get("align_corners", True), "align_mode": at.get("align_mode", 1),
                           "data_layout": at.get("data_layout", "NCHW")}, "Out"
    return conv


# ---------------------------------------------------------- data-dependent / stateful ops (round 5)
def unique_sorted_op(x, dtype=3, return_index=False, return_inverse=False, return_counts=False, axis=()):
    """unique_op.cc with is_sorted (paddle.unique): Out [+ Indices, Index, Counts as requested]"""
    from ..tensor.manipulation import unique
    r = unique(_wrap(_t(x)), return_index, return_inverse, return_counts, axis[0] if axis else None,
               pb.dtype_of(dtype) if dtype is not None and dtype >= 0 else "int64")
    return r


def unique_v1_op(x, dtype=2):
    """unique_op.cc without is_sorted (fluid.layers.unique): first-occurrence order, (Out, Index)"""
    from ..fluid.layers.nn import unique
    return unique(_wrap(_t(x)), pb.dtype_of(dtype) if dtype is not None and dtype >= 0 else "int32")


def _conv_unique(r, ins, at):
    if not at.get("is_sorted", False):
        return unique_v1_op, {"x": _one(r, ins, "X"), "dtype": at.get("dtype", 2)}, ("Out", "Index")
    outs = ["Out"] + [sl for f, sl in (("return_index", "Indices"), ("return_inverse", "Index"),
                                        ("return_counts", "Counts")) if at.get(f)]
    kw = {"x": _one(r, ins, "X"), "dtype": at.get("dtype", 3), "return_index": at.get("return_index", False),
          "return_inverse": at.get("return_inverse", False), "return_counts": at.get("return_counts", False),
          "axis": at.get("axis", [])}
    return unique_sorted_op, kw, tuple(outs) if len(outs) > 1 else "Out"


def accuracy_op(indices, label):
    """accuracy_op.cc on the top-k indices: (Accuracy [1] fp32, Correct [1] int32, Total [1] int32)"""
    idx = _t(indices)
    y = _t(label).reshape(-1, 1).long().to(idx.device)
    hit = (idx.long() == y).any(-1)
    n_ok = hit.sum().reshape(1)
    n = hit.numel()
    return (_wrap(n_ok.float() / max(n, 1)), _wrap(n_ok.int()),
            _wrap(torch.tensor([n], dtype=torch.int32, device=idx.device)))


def auc_ref_op(predict, label, stat_pos, stat_neg, num_thresholds=2 ** 12 - 1, slide_steps=1, curve="ROC"):
    from ..fluid.layers.metric_op import auc_op
    return auc_op(predict, label, stat_pos, stat_neg, num_thresholds, slide_steps, curve)


def _conv_print(r, ins, at):
    from ..fluid.layers.control_flow import _Printer
    x = _one(r, ins, "In")
    pr = _Printer(x.name if x is not None else None, at.get("first_n", -1), at.get("message", ""),
                  at.get("summarize", 20), at.get("print_tensor_name", True), at.get("print_tensor_type", True),
                  at.get("print_tensor_shape", True), at.get("print_tensor_lod", True),
                  str(at.get("print_phase", "BOTH")).lower())

    def print_op(x):
        return pr(x)
    return print_op, {"x": x}, "Out"


def lstm_ref_op(input, weight, bias, h0=None, c0=None, use_peepholes=True, is_reverse=False,
                gate_activation="sigmoid", cell_activation="tanh", candidate_activation="tanh"):
    """lstm_op.cc (LoD input [T, 4D] already projected; gates {c, i, f, o}; peephole weights in
    the bias tail) -> (Hidden, Cell)"""
    from ..fluid.layers.rnn import _lstm_run
    return _lstm_run(input, int(_t(weight).shape[0]), weight, bias, None, use_peepholes, is_reverse,
                     gate_activation, cell_activation, candidate_activation, h0, c0, None)


def gru_ref_op(input, weight, bias=None, h0=None, activation="tanh", gate_activation="sigmoid", is_reverse=False,
               origin_mode=False):
    """gru_op.cc (LoD input [T, 3D] already projected) -> Hidden"""
    from ..fluid.layers.rnn import _gru_run
    H = int(_t(weight).shape[0])
    b = bias if bias is not None else _wrap(torch.zeros(1, 3 * H, device=_t(weight).device))
    return _gru_run(input, weight, b, H, is_reverse, gate_activation, activation, h0, origin_mode)


def edit_distance_ref_op(hyps, refs, hyps_length=None, refs_length=None, normalized=False):
    from ..fluid.layers.loss import edit_distance
    return edit_distance(hyps, refs, normalized, None, hyps_length, refs_length)


def _kw(fn, slots, attrs, out, **fixed):
    """generic converter: slots {kwarg: input slot}, attrs {kwarg: (attr name, default)}"""
    def conv(r, ins, at):
        kw = {k: _one(r, ins, s) for k, s in slots.items()}
        kw.update({k: at.get(a, d) for k, (a, d) in attrs.items()})
        kw.update(fixed)
        return fn, kw, out
    return conv


def _conv_resnet_unit(r, ins, at):
    from ..incubate.operators.resnet_unit import resnet_unit
    slots = {"x": "X", "filter_x": "FilterX", "scale_x": "ScaleX", "bias_x": "BiasX", "mean_x": "MeanX",
             "var_x": "VarX", "z": "Z", "filter_z": "FilterZ", "scale_z": "ScaleZ", "bias_z": "BiasZ",
             "mean_z": "MeanZ", "var_z": "VarZ"}
    kw = {k: _one(r, ins, s) for k, s in slots.items()}
    kw.update(stride=at.get("stride", 1), stride_z=at.get("stride_z", 1), padding=at.get("padding", 0),
              dilation=at.get("dilation", 1), groups=at.get("group", 1), momentum=at.get("momentum", 0.9),
              eps=at.get("epsilon", 1e-5), data_format=at.get("data_format", "NHWC"),
              fuse_add=at.get("fuse_add", False), has_shortcut=at.get("has_shortcut", False),
              use_global_stats=at.get("use_global_stats", False), is_test=at.get("is_test", False),
              act=at.get("act_type", "relu"))
    return resnet_unit, kw, "Y"


def _conv_rnn(r, ins, at):
    """rnn_op.cc: Input, PreState, WeightList, SequenceLength -> Out, State (Reserve / DropoutState
    are the cuDNN workspace and dropout state: not produced here)"""
    from ..nn.functional.rnn_op import rnn_op
    kw = {"input": _one(r, ins, "Input"), "pre_state": _many(r, ins, "PreState"),
          "weight_list": _many(r, ins, "WeightList"), "sequence_length": _one(r, ins, "SequenceLength"),
          "dropout_prob": at.get("dropout_prob", 0.0), "is_bidirec": at.get("is_bidirec", False),
          "input_size": at.get("input_size", 10), "hidden_size": at.get("hidden_size", 100),
          "num_layers": at.get("num_layers", 1), "mode": at.get("mode", "LSTM"), "is_test": at.get("is_test", False)}
    return rnn_op, kw, ("Out", "State*")


def _conv_stack(r, ins, at):
    return stack_op, {"xs": _many(r, ins, "X"), "axis": at.get("axis", 0)}, "Y"


def _conv_unstack(r, ins, at):
    return unstack_op, {"x": _one(r, ins, "X"), "axis": at.get("axis", 0)}, ("list", "Y")


def _conv_split(r, ins, at):
    return split_op, {"x": _one(r, ins, "X"), "num": at.get("num", 0), "sections": at.get("sections", []),
                      "axis": at.get("axis", 0)}, ("list", "Out")


def _conv_sum(r, ins, at):
    return sum_op, {"xs": _many(r, ins, "X")}, "Out"


def _conv_meshgrid(r, ins, at):
    return meshgrid_op, {"xs": _many(r, ins, "X")}, ("list", "Out")


def _conv_assign_value(r, ins, at):
    vals = at.get("fp32_values") or at.get("int32_values") or at.get("int64_values") or at.get("bool_values") or []
    return assign_value_op, {"shape": at["shape"], "dtype": at.get("dtype", 5), "values": vals}, "Out"


def _conv_expand_as(r, ins, at):
    y = _one(r, ins, "Y")
    shape = at.get("target_shape") or (list(y.shape) if y is not None else [])
    return expand_as_op, {"x": _one(r, ins, "X"), "target_shape": shape}, "Out"


def _conv_gather(r, ins, at):
    return gather_op, {"x": _one(r, ins, "X"), "index": _one(r, ins, "Index"), "axis": at.get("axis", 0)}, "Out"


def _conv_conv_t(r, ins, at):
    return conv_transpose_op, {"x": _one(r, ins, "Input"), "weight": _one(r, ins, "Filter"),
                               "bias": _one(r, ins, "Bias"), "strides": at.get("strides", [1, 1]),
                               "paddings": at.get("paddings", [0, 0]), "dilations": at.get("dilations", [1, 1]),
                               "groups": at.get("groups", 1), "output_size": at.get("output_size", []),
                               "data_format": at.get("data_format", "NCHW"),
                               "padding_algorithm": at.get("padding_algorithm", "EXPLICIT")}, "Output"


def _conv_fluid(name, slots, attrs, out):
    def conv(r, ins, at):
        kw = {k: _one(r, ins, s) for k, s in slots.items()}
        kw.update({k: at.get(a, d) for k, (a, d) in attrs.items()})
        return _fluid(name), kw, out
    return conv


def _quant(name):
    from ..nn.quant import ops as QO
    return getattr(QO, name)


def _conv_q_absmax(typ):
    def conv(r, ins, at):
        return _quant(typ), {"x": _one(r, ins, "X"), "bit_length": at.get("bit_length", 8),
                             "round_type": at.get("round_type", 1)}, ("Out", "OutScale")
    return conv


def _conv_q_channel(typ):
    def conv(r, ins, at):
        return _quant(typ), {"x": _one(r, ins, "X"), "bit_length": at.get("bit_length", 8),
                             "quant_axis": at.get("quant_axis", 0), "round_type": at.get("round_type", 1)}, \
            ("Out", "OutScale")
    return conv


def _conv_q_channel_frozen(r, ins, at):
    """the channel-wise quant-dequant with a stored per-channel scale (our frozen weight form)"""
    if not ins.get("InScale"):
        return _conv_q_channel("fake_channel_wise_quantize_dequantize_abs_max")(r, ins, at)
    return _quant("fake_quantize_dequantize_fixed_scale"), {
        "x": _one(r, ins, "X"), "scale": _one(r, ins, "InScale"), "bit_length": at.get("bit_length", 8),
        "round_type": at.get("round_type", 1), "quant_axis": at.get("quant_axis", 0)}, "Out"


def _conv_q_moving(typ):
    def conv(r, ins, at):
        return _quant(typ), {"x": _one(r, ins, "X"), "in_scale": _one(r, ins, "InScale"),
                             "in_state": _one(r, ins, "InState"), "in_accum": _one(r, ins, "InAccum"),
                             "bit_length": at.get("bit_length", 8), "moving_rate": at.get("moving_rate", 0.9),
                             "is_test": at.get("is_test", True), "round_type": at.get("round_type", 1)}, "Out"
    return conv


def _conv_ma_scale(r, ins, at):
    return _quant("moving_average_abs_max_scale"), {
        "x": _one(r, ins, "X"), "in_scale": _one(r, ins, "InScale") or r.var(ins.get("OutScale", ["_"])[0]),
        "in_state": _one(r, ins, "InState"), "in_accum": _one(r, ins, "InAccum"),
        "moving_rate": at.get("moving_rate", 0.9), "is_test": at.get("is_test", True)}, "Out"


def _conv_q_linear(typ):
    def conv(r, ins, at):
        kw = {"x": _one(r, ins, "X"), "scale": _one(r, ins, "Scale"), "zero_point": _one(r, ins, "ZeroPoint"),
              "bit_length": at.get("bit_length", 8), "quant_axis": at.get("quant_axis", -1)}
        if typ == "quantize_linear":
            kw["round_type"] = at.get("round_type", 0)
        return _quant(typ), kw, "Y"
    return conv


# LoD sequence ops (sequence_ops/sequence_*_op.cc), run by fluid.layers.sequence_lod at run time
def _seq(name):
    from ..fluid.layers import sequence_lod as S
    f = getattr(S, name)
    return getattr(f, "__wrapped_op__", f)


def _conv_seq_pool(r, ins, at):
    return _seq("sequence_pool"), {"input": _one(r, ins, "X"), "pool_type": at.get("pooltype", "AVERAGE").lower(),
                                   "is_test": at.get("is_test", False), "pad_value": at.get("pad_value", 0.0)}, "Out"


def _conv_seq_conv(r, ins, at):
    return _seq("sequence_conv_op"), {"input": _one(r, ins, "X"), "filter": _one(r, ins, "Filter"),
                                      "context_length": at.get("contextLength", 3),
                                      "context_start": at.get("contextStart", -1),
                                      "context_stride": at.get("contextStride", 1)}, "Out"


def _conv_seq_pad(r, ins, at):
    pl = at.get("padded_length", -1)
    return _seq("sequence_pad"), {"x": _one(r, ins, "X"), "pad_value": _one(r, ins, "PadValue"),
                                  "maxlen": None if pl == -1 else pl}, ("Out", "Length")


def _conv_seq_mask(r, ins, at):
    ml = at.get("maxlen", -1)
    return _seq("sequence_mask"), {"x": _one(r, ins, "X"), "maxlen": None if ml == -1 else ml,
                                   "dtype": pb.dtype_of(at.get("out_dtype", 3))}, "Y"


_SEQ_CONVERT = {
    "sequence_pool": _conv_seq_pool,
    "sequence_conv": _conv_seq_conv,
    "sequence_softmax": lambda r, ins, at: (_seq("sequence_softmax"), {"input": _one(r, ins, "X")}, "Out"),
    "sequence_expand": lambda r, ins, at: (_seq("sequence_expand"), {"x": _one(r, ins, "X"), "y": _one(r, ins, "Y"),
                                                                     "ref_level": at.get("ref_level", -1)}, "Out"),
    "sequence_expand_as": lambda r, ins, at: (_seq("sequence_expand_as"), {"x": _one(r, ins, "X"),
                                                                           "y": _one(r, ins, "Y")}, "Out"),
    "sequence_pad": _conv_seq_pad,
    "sequence_unpad": lambda r, ins, at: (_seq("sequence_unpad"), {"x": _one(r, ins, "X"),
                                                                   "length": _one(r, ins, "Length")}, "Out"),
    "sequence_reverse": lambda r, ins, at: (_seq("sequence_reverse"), {"x": _one(r, ins, "X")}, "Y"),
    "sequence_concat": lambda r, ins, at: (_seq("sequence_concat"), {"input": _many(r, ins, "X")}, "Out"),
    "sequence_reshape": lambda r, ins, at: (_seq("sequence_reshape"), {"input": _one(r, ins, "X"),
                                                                       "new_dim": at["new_dim"]}, "Out"),
    "sequence_mask": _conv_seq_mask,
    "sequence_enumerate": lambda r, ins, at: (_seq("sequence_enumerate"), {
        "input": _one(r, ins, "X"), "win_size": at["win_size"], "pad_value": at.get("pad_value", 0)}, "Out"),
    "sequence_slice": lambda r, ins, at: (_seq("sequence_slice"), {
        "input": _one(r, ins, "X"), "offset": _one(r, ins, "Offset"), "length": _one(r, ins, "Length")}, "Out"),
    "sequence_scatter": lambda r, ins, at: (_seq("sequence_scatter"), {
        "input": _one(r, ins, "X"), "index": _one(r, ins, "Ids"), "updates": _one(r, ins, "Updates")}, "Out"),
}


CONVERT = {
    **_SEQ_CONVERT,
    # fake quantization (fake_quantize_op.cc, fake_dequantize_op.cc, quantize_linear_op.cc)
    "fake_quantize_dequantize_abs_max": _conv_q_absmax("fake_quantize_dequantize_abs_max"),
    "fake_quantize_abs_max": _conv_q_absmax("fake_quantize_abs_max"),
    "fake_channel_wise_quantize_dequantize_abs_max": _conv_q_channel_frozen,
    "fake_channel_wise_quantize_abs_max": _conv_q_channel("fake_channel_wise_quantize_abs_max"),
    "fake_quantize_dequantize_moving_average_abs_max": _conv_q_moving("fake_quantize_dequantize_moving_average_abs_max"),
    "fake_quantize_moving_average_abs_max": _conv_q_moving("fake_quantize_moving_average_abs_max"),
    "moving_average_abs_max_scale": _conv_ma_scale,
    "quantize_linear": _conv_q_linear("quantize_linear"),
    "dequantize_linear": _conv_q_linear("dequantize_linear"),
    "fake_dequantize_max_abs": lambda r, ins, at: (_quant("fake_dequantize_max_abs"), {
        "x": _one(r, ins, "X"), "scale": _one(r, ins, "Scale"), "max_range": at.get("max_range", 127.0)}, "Out"),
    "fake_channel_wise_dequantize_max_abs": lambda r, ins, at: (_quant("fake_channel_wise_dequantize_max_abs"), {
        "x": _one(r, ins, "X"), "scales": _one(r, ins, "Scales"), "quant_bits": at.get("quant_bits", [8]),
        "quant_axis": at.get("quant_axis", 0)}, "Out"),
    # activations / unary
    **{op: _unary(op) for op in ("abs", "acos", "asin", "atan", "ceil", "cos", "cosh", "floor", "log", "log1p", "log2",
                                 "log10", "reciprocal", "round", "rsqrt", "sin", "sinh", "square", "tan", "softsign",
                                 "expm1", "erf", "sign", "logsigmoid", "tanh_shrink", "logical_not", "isfinite_v2",
                                 "isnan_v2", "isinf_v2", "squared_l2_norm", "mean", "fill_zeros_like", "assign",
                                 "mish")},
    "relu6": _unary("relu6", threshold=6.0),
    "leaky_relu": _unary("leaky_relu", alpha=0.02),
    "elu": _unary("elu", alpha=1.0),
    "selu": _unary("selu", scale=1.0507009873554805, alpha=1.6732632423543772),
    "swish": _unary("swish", beta=1.0),
    "hard_swish": _unary("hard_swish", threshold=6.0, scale=6.0, offset=3.0),
    "hard_sigmoid": _unary("hard_sigmoid", slope=0.2, offset=0.5),
    "softshrink": _unary("softshrink", **{"lambda": 0.5}),
    "hard_shrink": _unary("hard_shrink", threshold=0.5),
    "thresholded_relu": _unary("thresholded_relu", threshold=1.0),
    "brelu": _unary("brelu", t_min=0.0, t_max=24.0),
    "stanh": _unary("stanh", scale_a=0.67, scale_b=1.7159),
    "soft_relu": _unary("soft_relu", threshold=40.0),
    "softplus": _unary("softplus", beta=1.0, threshold=20.0),
    "log_softmax": _unary("log_softmax", axis=-1),
    "prelu": _kw(prelu_op, {"x": "X", "alpha": "Alpha"}, {"mode": ("mode", "all"),
                                                          "data_format": ("data_format", "NCHW")}, "Out"),
    # binary / comparison / logic
    **{op: _binary(op) for op in ("elementwise_mod", "elementwise_floordiv", "less_than", "less_equal", "greater_than",
                                  "greater_equal", "equal", "not_equal", "logical_and", "logical_or", "logical_xor",
                                  "bmm", "dot")},
    "matmul": _kw(matmul_v1, {"x": "X", "y": "Y"}, {"transpose_X": ("transpose_X", False),
                                                    "transpose_Y": ("transpose_Y", False), "alpha": ("alpha", 1.0)},
                  "Out"),
    # shape / indexing
    "stack": _conv_stack,
    "resnet_unit": _conv_resnet_unit,
    "rnn": _conv_rnn,
    "unstack": _conv_unstack,
    "split": _conv_split,
    "gather": _conv_gather,
    "gather_nd": _kw(gather_nd_op, {"x": "X", "index": "Index"}, {}, "Out"),
    "shape": _kw(shape_op, {"x": "Input"}, {}, "Out"),
    "size": _kw(size_op, {"x": "Input"}, {}, "Out"),
    "expand_v2": _kw(expand_v2_op, {"x": "X"}, {"shape": ("shape", [])}, "Out"),
    "expand": _kw(expand_op, {"x": "X"}, {"expand_times": ("expand_times", [])}, "Out"),
    "expand_as_v2": _conv_expand_as,
    "tile": _kw(tile_op, {"x": "X"}, {"repeat_times": ("repeat_times", [])}, "Out"),
    "flatten2": _kw(flatten2_op, {"x": "X"}, {"axis": ("axis", 1)}, "Out"),
    "flatten": _kw(flatten2_op, {"x": "X"}, {"axis": ("axis", 1)}, "Out"),
    "reshape": _kw(reshape_v1, {"x": "X"}, {"shape": ("shape", [])}, "Out"),
    "transpose": _kw(transpose_v1, {"x": "X"}, {"axis": ("axis", [])}, "Out"),
    "squeeze": _kw(squeeze_v1, {"x": "X"}, {"axes": ("axes", [])}, "Out"),
    "unsqueeze": _kw(unsqueeze_v1, {"x": "X"}, {"axes": ("axes", [])}, "Out"),
    "arg_max": _kw(arg_op, {"x": "X"}, {"axis": ("axis", -1), "keepdims": ("keepdims", False),
                                        "flatten": ("flatten", False), "dtype": ("dtype", 3)}, "Out", op="arg_max"),
    "arg_min": _kw(arg_op, {"x": "X"}, {"axis": ("axis", -1), "keepdims": ("keepdims", False),
                                        "flatten": ("flatten", False), "dtype": ("dtype", 3)}, "Out", op="arg_min"),
    "top_k": _kw(top_k_op, {"x": "X"}, {"k": ("k", 1)}, ("Out", "Indices")),
    "top_k_v2": _kw(top_k_op, {"x": "X"}, {"k": ("k", 1), "axis": ("axis", -1), "largest": ("largest", True),
                                           "sorted": ("sorted", True)}, ("Out", "Indices")),
    "argsort": _kw(argsort_op, {"x": "X"}, {"axis": ("axis", -1), "descending": ("descending", False)},
                   ("Out", "Indices")),
    "cumsum": _kw(cumsum_op, {"x": "X"}, {"axis": ("axis", -1), "exclusive": ("exclusive", False),
                                          "reverse": ("reverse", False), "flatten": ("flatten", False)}, "Out"),
    "clip": _kw(clip_op, {"x": "X"}, {"min": ("min", -3.4e38), "max": ("max", 3.4e38)}, "Out"),
    "where": _kw(where_op, {"condition": "Condition", "x": "X", "y": "Y"}, {}, "Out"),
    "where_index": _kw(where_index_op, {"condition": "Condition"}, {}, "Out"),
    "unique": _conv_unique,
    "accuracy": _kw(accuracy_op, {"indices": "Indices", "label": "Label"}, {}, ("Accuracy", "Correct", "Total")),
    "auc": _kw(auc_ref_op, {"predict": "Predict", "label": "Label", "stat_pos": "StatPos", "stat_neg": "StatNeg"},
               {"num_thresholds": ("num_thresholds", 2 ** 12 - 1), "slide_steps": ("slide_steps", 1),
                "curve": ("curve", "ROC")}, "AUC"),
    "print": _conv_print,
    "lstm": _kw(lstm_ref_op, {"input": "Input", "weight": "Weight", "bias": "Bias", "h0": "H0", "c0": "C0"},
                {"use_peepholes": ("use_peepholes", True), "is_reverse": ("is_reverse", False),
                 "gate_activation": ("gate_activation", "sigmoid"), "cell_activation": ("cell_activation", "tanh"),
                 "candidate_activation": ("candidate_activation", "tanh")}, ("Hidden", "Cell")),
    "gru": _kw(gru_ref_op, {"input": "Input", "weight": "Weight", "bias": "Bias", "h0": "H0"},
               {"activation": ("activation", "tanh"), "gate_activation": ("gate_activation", "sigmoid"),
                "is_reverse": ("is_reverse", False), "origin_mode": ("origin_mode", False)}, "Hidden"),
    "edit_distance": _kw(edit_distance_ref_op, {"hyps": "Hyps", "refs": "Refs", "hyps_length": "HypsLength",
                                                "refs_length": "RefsLength"},
                         {"normalized": ("normalized", False)}, ("Out", "SequenceNum")),
    "one_hot_v2": _kw(one_hot_op, {"x": "X"}, {"depth": ("depth", 1)}, "Out"),
    "one_hot": _kw(one_hot_op, {"x": "X"}, {"depth": ("depth", 1)}, "Out", v1=True),
    "range": _kw(range_op, {"start": "Start", "end": "End", "step": "Step"}, {}, "Out"),
    "linspace": _kw(linspace_op, {"start": "Start", "stop": "Stop", "num": "Num"}, {"dtype": ("dtype", 5)}, "Out"),
    "fill_any_like": _kw(fill_any_like_op, {"x": "X"}, {"value": ("value", 0.0), "dtype": ("dtype", -1)}, "Out"),
    "fill_constant_batch_size_like": _kw(fill_constant_bsl_op, {"input": "Input"},
                                         {"shape": ("shape", []), "value": ("value", 0.0), "dtype": ("dtype", 5),
                                          "input_dim_idx": ("input_dim_idx", 0),
                                          "output_dim_idx": ("output_dim_idx", 0)}, "Out"),
    "assign_value": _conv_assign_value,
    "pad": _kw(pad_op, {"x": "X"}, {"paddings": ("paddings", []), "pad_value": ("pad_value", 0.0)}, "Out"),
    "pad2d": _kw(pad_nd_op, {"x": "X"}, {"paddings": ("paddings", [0, 0, 0, 0]), "mode": ("mode", "constant"),
                                         "value": ("pad_value", 0.0), "data_format": ("data_format", "NCHW")}, "Out"),
    "pad3d": _kw(pad_nd_op, {"x": "X"}, {"paddings": ("paddings", [0] * 6), "mode": ("mode", "constant"),
                                         "value": ("value", 0.0), "data_format": ("data_format", "NCDHW")}, "Out"),
    "strided_slice": _kw(strided_slice_op, {"x": "Input"}, {"axes": ("axes", []), "starts": ("starts", []),
                                                            "ends": ("ends", []), "strides": ("strides", []),
                                                            "decrease_axis": ("decrease_axis", [])}, "Out"),
    "index_select": _kw(index_select_op, {"x": "X", "index": "Index"}, {"dim": ("dim", 0)}, "Out"),
    "scatter": _kw(scatter_op, {"x": "X", "ids": "Ids", "updates": "Updates"}, {"overwrite": ("overwrite", True)},
                   "Out"),
    "tril_triu": _kw(tril_triu_op, {"x": "X"}, {"diagonal": ("diagonal", 0), "lower": ("lower", False)}, "Out"),
    "masked_select": _kw(masked_select_op, {"x": "X", "mask": "Mask"}, {}, "Y"),
    "meshgrid": _conv_meshgrid,
    "roll": _kw(roll_op, {"x": "X"}, {"shifts": ("shifts", []), "axis": ("axis", [])}, "Out"),
    "flip": _kw(flip_op, {"x": "X"}, {"axis": ("axis", [])}, "Out"),
    "sum": _conv_sum,
    # interpolation / vision
    "bilinear_interp_v2": _interp("bilinear"), "nearest_interp_v2": _interp("nearest"),
    "linear_interp_v2": _interp("linear"), "bicubic_interp_v2": _interp("bicubic"),
    "trilinear_interp_v2": _interp("trilinear"), "bilinear_interp": _interp("bilinear"),
    "nearest_interp": _interp("nearest"),
    "pixel_shuffle": _kw(pixel_shuffle_op, {"x": "X"}, {"upscale_factor": ("upscale_factor", 1),
                                                        "data_format": ("data_format", "NCHW")}, "Out"),
    "shuffle_channel": _kw(shuffle_channel_op, {"x": "X"}, {"group": ("group", 1)}, "Out"),
    "affine_channel": _kw(affine_channel_op, {"x": "X", "scale": "Scale", "bias": "Bias"},
                          {"data_layout": ("data_layout", "NCHW")}, "Out"),
    "conv2d_transpose": _conv_conv_t,
    "conv3d_transpose": _conv_conv_t,
    "conv3d": _kw(conv3d_op, {"x": "Input", "weight": "Filter", "bias": "Bias"},
                  {"strides": ("strides", [1, 1, 1]), "paddings": ("paddings", [0, 0, 0]),
                   "dilations": ("dilations", [1, 1, 1]), "groups": ("groups", 1),
                   "data_format": ("data_format", "NCDHW")}, "Output"),
    "pool3d": _kw(pool3d_op, {"x": "X"}, {"pooling_type": ("pooling_type", "max"), "ksize": ("ksize", [1, 1, 1]),
                                          "strides": ("strides", [1, 1, 1]), "paddings": ("paddings", [0, 0, 0]),
                                          "global_pooling": ("global_pooling", False),
                                          "exclusive": ("exclusive", True), "ceil_mode": ("ceil_mode", False)}, "Out"),
    "instance_norm": _kw(instance_norm_op, {"x": "X", "scale": "Scale", "bias": "Bias"},
                         {"epsilon": ("epsilon", 1e-5)}, "Y"),
    "group_norm": _kw(group_norm_op, {"x": "X", "scale": "Scale", "bias": "Bias"},
                      {"epsilon": ("epsilon", 1e-5), "groups": ("groups", 1), "data_layout": ("data_layout", "NCHW")},
                      "Y"),
    "reduce_min": _reduce("reduce_min"), "reduce_prod": _reduce("reduce_prod"),
    "reduce_all": _reduce("reduce_all"), "reduce_any": _reduce("reduce_any"),
    "p_norm": _kw(p_norm_op, {"x": "X"}, {"porder": ("porder", 2.0), "axis": ("axis", -1),
                                          "keepdim": ("keepdim", False), "epsilon": ("epsilon", 1e-12)}, "Out"),
    "norm": _kw(norm_op, {"x": "X"}, {"axis": ("axis", 1), "epsilon": ("epsilon", 1e-10)}, ("Out", "Norm")),
    "lookup_table": _kw(lookup_v1_op, {"ids": "Ids", "w": "W"}, {"padding_idx": ("padding_idx", -1)}, "Out"),
    "roi_align": _kw(roi_align_op, {"x": "X", "rois": "ROIs", "rois_num": "RoisNum"},
                     {"pooled_height": ("pooled_height", 1), "pooled_width": ("pooled_width", 1),
                      "spatial_scale": ("spatial_scale", 1.0), "sampling_ratio": ("sampling_ratio", -1),
                      "aligned": ("aligned", False)}, "Out"),
    "prior_box": _kw(prior_box_op, {"input": "Input", "image": "Image"},
                     {"min_sizes": ("min_sizes", []), "max_sizes": ("max_sizes", []),
                      "aspect_ratios": ("aspect_ratios", [1.0]), "variances": ("variances", [0.1, 0.1, 0.2, 0.2]),
                      "flip": ("flip", False), "clip": ("clip", False), "step_w": ("step_w", 0.0),
                      "step_h": ("step_h", 0.0), "offset": ("offset", 0.5),
                      "min_max_aspect_ratios_order": ("min_max_aspect_ratios_order", False)},
                     ("Boxes", "Variances")),
    "box_coder": _kw(box_coder_op, {"prior_box": "PriorBox", "prior_box_var": "PriorBoxVar",
                                    "target_box": "TargetBox"},
                     {"code_type": ("code_type", "encode_center_size"), "box_normalized": ("box_normalized", True),
                      "axis": ("axis", 0), "variance": ("variance", [])}, "OutputBox"),
    "multiclass_nms": _kw(multiclass_nms_op, {"bboxes": "BBoxes", "scores": "Scores"},
                          {"score_threshold": ("score_threshold", 0.05), "nms_top_k": ("nms_top_k", -1),
                           "keep_top_k": ("keep_top_k", -1), "nms_threshold": ("nms_threshold", 0.3),
                           "normalized": ("normalized", True), "nms_eta": ("nms_eta", 1.0),
                           "background_label": ("background_label", 0)}, "Out"),
    "yolo_box": _kw(yolo_box_op, {"x": "X", "img_size": "ImgSize"},
                    {"anchors": ("anchors", []), "class_num": ("class_num", 1), "conf_thresh": ("conf_thresh", 0.01),
                     "downsample_ratio": ("downsample_ratio", 32), "clip_bbox": ("clip_bbox", True),
                     "scale_x_y": ("scale_x_y", 1.0)}, ("Boxes", "Scores")),
    "uniform_random": _kw(random_op, {}, {"shape": ("shape", []), "min": ("min", -1.0), "max": ("max", 1.0),
                                          "seed": ("seed", 0), "dtype": ("dtype", 5)}, "Out", op="uniform_random"),
    "gaussian_random": _kw(random_op, {}, {"shape": ("shape", []), "mean": ("mean", 0.0), "std": ("std", 1.0),
                                           "seed": ("seed", 0), "dtype": ("dtype", 5)}, "Out", op="gaussian_random"),
    "grid_sampler": _kw(grid_sampler_op, {"x": "X", "grid": "Grid"},
                        {"align_corners": ("align_corners", True), "mode": ("mode", "bilinear"),
                         "padding_mode": ("padding_mode", "zeros")}, "Output"),
    "unfold": _kw(unfold_op, {"x": "X"}, {"kernel_sizes": ("kernel_sizes", [1, 1]), "strides": ("strides", [1, 1]),
                                          "paddings": ("paddings", [0, 0, 0, 0]),
                                          "dilations": ("dilations", [1, 1])}, "Y"),
    # 1.x layers with the same semantics as fluid.layers
    "maxout": _conv_fluid("maxout", {"x": "X"}, {"groups": ("groups", 1), "axis": ("axis", 1)}, "Out"),
    "lrn": _conv_fluid("lrn", {"input": "X"}, {"n": ("n", 5), "k": ("k", 1.0), "alpha": ("alpha", 1e-4),
                                               "beta": ("beta", 0.75), "data_format": ("data_format", "NCHW")},
                       "Out"),
    "space_to_depth": _conv_fluid("space_to_depth", {"x": "X"}, {"blocksize": ("blocksize", 1)}, "Out"),
    "temporal_shift": _conv_fluid("temporal_shift", {"x": "X"}, {"seg_num": ("seg_num", 1),
                                                                 "shift_ratio": ("shift_ratio", 0.25)}, "Out"),
    "crop_tensor": _conv_fluid("crop_tensor", {"x": "X"}, {"shape": ("shape", None), "offsets": ("offsets", None)},
                               "Out"),
    "affine_grid": _conv_fluid("affine_grid", {"theta": "Theta"}, {"out_shape": ("output_shape", [])}, "Output"),
    "increment": _conv_fluid("increment", {"x": "X"}, {"value": ("step", 1.0)}, "Out"),
}


# ----------------------------------------------------------------------------- control flow (1.x layout)
def _truth(v):
    return bool(_t(v).reshape(-1)[0].item())


def _exec_cond_block(program, env, op):
    from .program import run_block, _subst
    conds = op.kwargs["Cond"]
    if op.attrs["is_scalar_condition"]:
        take = _truth(_subst(conds[0], env))
    else:
        take = all(_t(_subst(c, env)).numel() > 0 for c in conds)
    if take:
        run_block(program, program.blocks[op.attrs["sub_block"]], env)


def _exec_while_v1(program, env, op):
    from .program import run_block
    c = op.kwargs["Condition"]
    body = program.blocks[op.attrs["sub_block"]]
    n = 0
    while _truth(env[id(c)]):
        run_block(program, body, env)
        n += 1
        if n > 10_000_000:
            raise RuntimeError("while: more than 1e7 iterations")


def select_input_op(xs, mask):
    return xs[int(_t(mask).reshape(-1)[0].item())]


def write_to_array_op(arr, x, i):
    out = list(arr) if isinstance(arr, list) else []
    k = int(_t(i).reshape(-1)[0].item())
    while len(out) <= k:
        out.append(None)
    out[k] = x
    return out


def read_from_array_op(arr, i):
    return arr[int(_t(i).reshape(-1)[0].item())]


def array_length_op(arr):
    return _wrap(torch.tensor([len(arr) if isinstance(arr, list) else 0], dtype=torch.int64,
                              device=_core.default_device()))


def _cf_conditional_block(r, blk, ins, outs, at):
    from .program import OpDesc
    from .control_flow import _captured
    sub = r.prog.blocks[at["sub_block"]]
    written = [r.var(n) for n in outs.get("Out", [])]
    return OpDesc("conditional_block", None, (), {"Cond": [r.var(n) for n in ins.get("Cond", [])],
                                                  "Input": [r.var(n) for n in ins.get("Input", [])]}, written,
                  attrs={"sub_block": at["sub_block"], "is_scalar_condition": at.get("is_scalar_condition", False),
                         "captured": _captured([sub]), "ref_layout": True}, exec=_exec_cond_block)


def _cf_while(r, blk, ins, outs, at):
    from .program import OpDesc
    from .control_flow import _captured
    sub = r.prog.blocks[at["sub_block"]]
    cond = r.var(ins["Condition"][0])
    return OpDesc("while", None, (), {"Condition": cond, "X": [r.var(n) for n in ins.get("X", [])]},
                  [r.var(n) for n in outs.get("Out", [])],
                  attrs={"sub_block": at["sub_block"], "captured": _captured([sub]) + [cond], "ref_layout": True},
                  exec=_exec_while_v1)


def _exec_write_to_array(program, env, op):
    from .program import _subst
    arr = op.kwargs["Out"]
    env[id(arr)] = write_to_array_op(env.get(id(arr), []), _subst(op.kwargs["X"], env), _subst(op.kwargs["I"], env))


def _cf_write_to_array(r, blk, ins, outs, at):
    from .program import OpDesc
    arr = r.var(outs["Out"][0])
    return OpDesc("write_to_array", None, (), {"X": r.var(ins["X"][0]), "I": r.var(ins["I"][0]), "Out": arr}, [],
                  attrs={"captured": [arr]}, exec=_exec_write_to_array)


CF = {"conditional_block": _cf_conditional_block, "while": _cf_while, "write_to_array": _cf_write_to_array}

CONVERT.update({
    "select_input": lambda r, ins, at: (select_input_op, {"xs": _many(r, ins, "X"), "mask": _one(r, ins, "Mask")},
                                        "Out"),
    "read_from_array": lambda r, ins, at: (read_from_array_op, {"arr": _one(r, ins, "X"), "i": _one(r, ins, "I")},
                                           "Out"),
    "lod_array_length": lambda r, ins, at: (array_length_op, {"arr": _one(r, ins, "X")}, "Out"),
})
