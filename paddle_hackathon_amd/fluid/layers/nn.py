"""``fluid.layers`` neural-network layers with the 1.x signatures and semantics (reference:
python/paddle/fluid/layers/nn.py; the op definitions they call live under
paddle/fluid/operators/*_op.{cc,h}). Every function works on dygraph Tensors and, in static mode,
records one op of its fluid type (``elementwise_add``, ``reduce_sum`` ...) into the current
Program. Parameter-creating builders (fc, conv2d, batch_norm ...) create their parameters and
then emit functional ops, like ``paddle.static.nn``.

Where 1.x semantics differ from 2.x they follow 1.x: ``dropout`` defaults to
``downgrade_in_infer``, ``one_hot`` / ``embedding`` consume a trailing unit dimension,
``flatten`` produces 2-D, ``lrn`` does not divide alpha by n, resize ops default to
``align_corners=True``, ``where`` returns coordinates.
"""
from __future__ import annotations

import builtins as _b
import math

import numpy as np
import torch
import torch.nn.functional as TF

from ...framework.core import Tensor
from ...nn import functional as F
from ... import static as _static
from ...static import nn as SN
from ._common import T, W, dt, dev, act, bcast_y, norm_axes, write_to, to_padded, from_padded, register
from .. import core as fcore

builtins_slice = _b.slice

__all__ = [
    "fc", "embedding", "linear_chain_crf", "crf_decoding", "cos_sim", "chunk_eval", "conv2d", "conv3d", "softmax",
    "pool2d", "pool3d", "adaptive_pool2d", "adaptive_pool3d", "batch_norm", "inplace_abn", "instance_norm",
    "data_norm", "conv2d_transpose", "conv3d_transpose", "reduce_sum", "reduce_mean", "reduce_max", "reduce_min",
    "reduce_prod", "reduce_all", "reduce_any", "dropout", "split", "ctc_greedy_decoder", "l2_normalize", "matmul",
    "topk", "transpose", "im2sequence", "row_conv", "multiplex", "layer_norm", "group_norm", "spectral_norm",
    "smooth_l1", "one_hot", "autoincreased_step_counter", "reshape", "squeeze", "unsqueeze", "lod_reset",
    "lod_append", "lrn", "pad", "pad_constant_like", "label_smooth", "roi_pool", "roi_align", "dice_loss",
    "image_resize", "image_resize_short", "resize_linear", "resize_bilinear", "resize_trilinear", "resize_nearest",
    "gather", "gather_nd", "scatter", "scatter_nd_add", "scatter_nd", "random_crop", "mean_iou", "relu", "selu",
    "log", "crop", "crop_tensor", "elu", "relu6", "pow", "stanh", "hard_sigmoid", "swish", "prelu", "brelu",
    "leaky_relu", "soft_relu", "flatten", "stack", "pad2d", "unstack", "unique", "unique_with_counts", "expand",
    "expand_as", "scale", "elementwise_add", "elementwise_div", "elementwise_sub", "elementwise_mul",
    "elementwise_max", "elementwise_min", "elementwise_pow", "elementwise_mod", "elementwise_floordiv",
    "uniform_random_batch_size_like", "gaussian_random", "sampling_id", "gaussian_random_batch_size_like", "sum",
    "slice", "strided_slice", "shape", "rank", "size", "logical_and", "logical_or", "logical_xor", "logical_not",
    "clip", "clip_by_norm", "mean", "mul", "maxout", "space_to_depth", "affine_grid", "affine_channel",
    "similarity_focus", "hash", "grid_sampler", "log_loss", "add_position_encoding", "bilinear_tensor_product",
    "merge_selected_rows", "get_tensor_from_selected_rows", "shuffle_channel", "temporal_shift", "py_func",
    "psroi_pool", "prroi_pool", "pixel_shuffle", "fsp_matrix", "continuous_value_model", "where", "sign",
    "deformable_conv", "unfold", "deformable_roi_pooling", "filter_by_instag", "shard_index", "hard_swish", "mish",
    "gather_tree", "uniform_random", "unbind",
]

# builders that create parameters or run Python callbacks: not recorded as a single op
_BUILDERS = {"fc", "embedding", "linear_chain_crf", "crf_decoding", "conv2d", "conv3d", "batch_norm", "inplace_abn",
             "instance_norm", "data_norm", "conv2d_transpose", "conv3d_transpose", "row_conv", "layer_norm",
             "group_norm", "spectral_norm", "prelu", "bilinear_tensor_product", "py_func", "deformable_conv",
             "autoincreased_step_counter", "affine_channel", "chunk_eval", "mean_iou", "similarity_focus", "hash",
             "logical_and", "logical_or", "logical_xor", "logical_not", "lod_reset", "lod_append"}
# (unique / unique_with_counts / where / filter_by_instag / sampling_id / random_crop /
# ctc_greedy_decoder / im2sequence record one op each: their data-dependent or host-read output
# shapes come from static/program.py's example-run InferMeta)


# ----------------------------------------------------------------------------- parameter builders
def fc(input, size, num_flatten_dims=1, param_attr=None, bias_attr=None, act=None, name=None):
    """``nn.py:fc`` — out = act(sum_i flatten(x_i) W_i + b)"""
    return SN.fc(input, size, num_flatten_dims, param_attr, bias_attr, act, name)


def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None, param_attr=None,
              dtype="float32"):
    """lookup_table (v1): ``input``'s last dimension must be 1 and is replaced by the embedding"""
    from ._common import fparam as _create_parameter
    from ...nn import initializer as I
    w = _create_parameter(list(size), dtype, param_attr, default_initializer=I.XavierUniform())
    if padding_idx is not None and padding_idx < 0:
        padding_idx += size[0]
    return _lookup_v1(input, w, padding_idx)


def _lookup_v1(input, w, padding_idx):
    ids = T(input)
    if ids.dim() > 1 and ids.shape[-1] == 1:
        ids = ids.squeeze(-1)
    out = TF.embedding(ids.long(), T(w), padding_idx=padding_idx)
    return W(out, input)


def conv2d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None, param_attr=None,
           bias_attr=None, use_cudnn=True, act=None, name=None, data_format="NCHW"):
    return SN.conv2d(input, num_filters, filter_size, stride, padding, dilation, groups, param_attr, bias_attr,
                     use_cudnn, act, name, data_format)


def conv3d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None, param_attr=None,
           bias_attr=None, use_cudnn=True, act=None, name=None, data_format="NCDHW"):
    return SN.conv3d(input, num_filters, filter_size, stride, padding, dilation, groups, param_attr, bias_attr,
                     use_cudnn, act, name, data_format)


def conv2d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,
                     groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
                     data_format="NCHW"):
    return SN.conv2d_transpose(input, num_filters, output_size, filter_size, padding, stride, dilation, groups,
                               param_attr, bias_attr, use_cudnn, act, name, data_format)


def conv3d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,
                     groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
                     data_format="NCDHW"):
    return SN.conv3d_transpose(input, num_filters, output_size, filter_size, padding, stride, dilation, groups,
                               param_attr, bias_attr, use_cudnn, act, name, data_format)


def batch_norm(input, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None, bias_attr=None,
               data_layout="NCHW", in_place=False, name=None, moving_mean_name=None, moving_variance_name=None,
               do_model_average_for_mean_and_var=True, use_global_stats=False):
    return SN.batch_norm(input, act, is_test, momentum, epsilon, param_attr, bias_attr, data_layout, in_place, name,
                         moving_mean_name, moving_variance_name, do_model_average_for_mean_and_var, use_global_stats)


def inplace_abn(input, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None, bias_attr=None,
                data_layout="NCHW", name=None, moving_mean_name=None, moving_variance_name=None,
                do_model_average_for_mean_and_var=True, use_global_stats=False, act_alpha=1.0):
    """batch_norm + identity / leaky_relu / elu activation (inplace_abn_op.cc)"""
    y = SN.batch_norm(input, None, is_test, momentum, epsilon, param_attr, bias_attr, data_layout, False, name,
                      moving_mean_name, moving_variance_name, do_model_average_for_mean_and_var, use_global_stats)
    if act == "leaky_relu":
        return F.leaky_relu(y, act_alpha)
    if act == "elu":
        return F.elu(y, act_alpha)
    if act in (None, "identity"):
        return y
    raise ValueError(f"inplace_abn: activation {act!r} (identity, leaky_relu, elu)")


def instance_norm(input, epsilon=1e-05, param_attr=None, bias_attr=None, name=None):
    return SN.instance_norm(input, epsilon, param_attr, bias_attr, name)


def data_norm(input, act=None, epsilon=1e-05, param_attr=None, data_layout="NCHW", in_place=False, name=None,
              moving_mean_name=None, moving_variance_name=None, do_model_average_for_mean_and_var=True,
              slot_dim=-1, sync_stats=False, summary_decay_rate=0.9999999, enable_scale_and_shift=False):
    return SN.data_norm(input, act, epsilon, param_attr, data_layout, in_place, name, moving_mean_name,
                        moving_variance_name, do_model_average_for_mean_and_var, slot_dim, sync_stats,
                        summary_decay_rate, enable_scale_and_shift)


def layer_norm(input, scale=True, shift=True, begin_norm_axis=1, epsilon=1e-05, param_attr=None, bias_attr=None,
               act=None, name=None):
    return SN.layer_norm(input, scale, shift, begin_norm_axis, epsilon, param_attr, bias_attr, act, name)


def group_norm(input, groups, epsilon=1e-05, param_attr=None, bias_attr=None, act=None, data_layout="NCHW",
               name=None):
    return SN.group_norm(input, groups, epsilon, param_attr, bias_attr, act, data_layout, name)


def spectral_norm(weight, dim=0, power_iters=1, eps=1e-12, name=None):
    return SN.spectral_norm(weight, dim, power_iters, eps, name)


def row_conv(input, future_context_size, param_attr=None, act=None):
    return SN.row_conv(input, future_context_size, param_attr, act)


def prelu(x, mode, param_attr=None, data_format="NCHW", name=None):
    return SN.prelu(x, mode, param_attr, data_format, name)


def bilinear_tensor_product(x, y, size, act=None, name=None, param_attr=None, bias_attr=None):
    return SN.bilinear_tensor_product(x, y, size, act, name, param_attr, bias_attr)


def deformable_conv(input, offset, mask, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None,
                    deformable_groups=None, im2col_step=None, param_attr=None, bias_attr=None, modulated=True,
                    name=None):
    return SN.deform_conv2d(input, offset, mask if modulated else None, num_filters, filter_size, stride, padding,
                            dilation, groups or 1, deformable_groups or 1, im2col_step or 1, param_attr, bias_attr,
                            name)


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    return _static.py_func(func, x, out, backward_func, skip_vars_in_backward_input)


def affine_channel(x, scale=None, bias=None, data_layout="NCHW", name=None, act=None):
    """out = x * scale[c] + bias[c] (affine_channel_op.cc)"""
    xt = T(x)
    c_axis = 1 if data_layout == "NCHW" else xt.dim() - 1
    shape = [1] * xt.dim()
    shape[c_axis] = xt.shape[c_axis]
    out = xt
    if scale is not None:
        out = out * T(scale).reshape(shape)
    if bias is not None:
        out = out + T(bias).reshape(shape)
    return act_(W(out), act)


act_ = act


# ----------------------------------------------------------------------------- CRF / sequence labelling
def _crf_transition(param_attr, size, dtype):
    from ._common import fparam
    return fparam([size + 2, size], dtype, param_attr)


def get_parameter(name):
    """a parameter created by a fluid builder (or recorded in the current Program), by name"""
    from ._common import _NAMED_PARAMS
    if name in _NAMED_PARAMS:
        return _NAMED_PARAMS[name]
    for p in _static.default_main_program().all_parameters():
        if p.name == name:
            return p
    raise ValueError(f"parameter {name!r} not found")


def linear_chain_crf(input, label, param_attr=None, length=None):
    """negative log-likelihood per sequence, [N, 1] (linear_chain_crf_op.h). Transition parameter
    rows: 0 = start weights, 1 = end weights, 2.. = tag-to-tag transitions."""
    size = input.shape[-1]
    trans = _crf_transition(param_attr, size, "float32")
    x, lens, lod = to_padded(input, length)
    y, _, _ = to_padded(label, length)
    y = y.reshape(y.shape[0], y.shape[1]).long()
    tw = T(trans)
    start, end, A = tw[0], tw[1], tw[2:]
    B, Tm, _ = x.shape
    m = torch.arange(Tm, device=x.device)[None, :] < lens[:, None].to(x.device)
    # log partition: forward algorithm over valid steps
    alpha = start[None, :] + x[:, 0]
    for t in range(1, Tm):
        nxt = torch.logsumexp(alpha[:, :, None] + A[None], dim=1) + x[:, t]
        alpha = torch.where(m[:, t:t + 1], nxt, alpha)
    logz = torch.logsumexp(alpha + end[None, :], dim=1)
    # gold path score
    idx = torch.arange(B, device=x.device)
    emit = (x.gather(2, y[:, :, None]).squeeze(2) * m).sum(1)
    tr = (A[y[:, :-1], y[:, 1:]] * m[:, 1:]).sum(1) if Tm > 1 else torch.zeros(B, device=x.device)
    last = y[idx, (lens.to(x.device) - 1).clamp_min(0)]
    gold = start[y[:, 0]] + emit + tr + end[last]
    return W((logz - gold)[:, None])


def crf_decoding(input, param_attr, label=None, length=None):
    """Viterbi path with the transition layout of linear_chain_crf (crf_decoding_op.h); with
    ``label`` it returns 1 where the decoded tag equals the label"""
    name = param_attr.name if hasattr(param_attr, "name") else param_attr
    tw = T(get_parameter(name))
    x, lens, lod = to_padded(input, length)
    start, end, A = tw[0], tw[1], tw[2:]
    B, Tm, K = x.shape
    paths = torch.zeros(B, Tm, dtype=torch.long, device=x.device)
    for b in range(B):
        n = int(lens[b])
        if n == 0:
            continue
        score = start + x[b, 0]
        back = []
        for t in range(1, n):
            s = score[:, None] + A
            best, arg = s.max(0)
            back.append(arg)
            score = best + x[b, t]
        score = score + end
        k = int(score.argmax())
        paths[b, n - 1] = k
        for t in range(n - 2, -1, -1):
            k = int(back[t][k])
            paths[b, t] = k
    if label is not None:
        y, _, _ = to_padded(label, length)
        paths = (paths == y.reshape(B, Tm).long()).long()
    if lod:
        return from_padded(paths[:, :, None], lens, fcore.lod_of(input))
    return W(paths)


def _chunks(tags, scheme, num_types, excluded):
    """(begin, end, type) spans of one tag sequence (chunk_eval_op.h)"""
    if scheme == "plain":
        out, i = [], 0
        while i < len(tags):
            t = tags[i]
            if t < num_types and t not in excluded:
                j = i
                while j + 1 < len(tags) and tags[j + 1] == t:
                    j += 1
                out.append((i, j, t))
                i = j + 1
            else:
                i += 1
        return out
    ntag = {"IOB": 2, "IOE": 2, "IOBES": 4}[scheme]
    other = num_types * ntag
    spans, start, ctype = [], None, None

    def close(end):
        if start is not None and ctype not in excluded:
            spans.append((start, end, ctype))

    for i, tag in enumerate(tags):
        if tag >= other or tag < 0:
            close(i - 1)
            start, ctype = None, None
            continue
        ty, pos = tag // ntag, tag % ntag
        if scheme == "IOB":
            if pos == 0 or ty != ctype or start is None:
                close(i - 1)
                start, ctype = i, ty
        elif scheme == "IOE":
            if start is None or ty != ctype:
                close(i - 1)
                start, ctype = i, ty
            if pos == 1:
                close(i)
                start, ctype = None, None
        else:   # IOBES: B=0 I=1 E=2 S=3
            if pos in (0, 3) or start is None or ty != ctype:
                close(i - 1)
                start, ctype = i, ty
            if pos in (2, 3):
                close(i)
                start, ctype = None, None
    close(len(tags) - 1)
    return spans


def chunk_eval(input, label, chunk_scheme, num_chunk_types, excluded_chunk_types=None, seq_length=None):
    """(precision, recall, f1, num_infer_chunks, num_label_chunks, num_correct_chunks)"""
    x, lens, _ = to_padded(input, seq_length)
    y, _, _ = to_padded(label, seq_length)
    x = x.reshape(x.shape[0], -1).cpu().tolist()
    y = y.reshape(y.shape[0], -1).cpu().tolist()
    ex = set(excluded_chunk_types or [])
    ni = nl = nc = 0
    for b, n in enumerate(lens.tolist()):
        pi = set(_chunks(x[b][:n], chunk_scheme, num_chunk_types, ex))
        pl = set(_chunks(y[b][:n], chunk_scheme, num_chunk_types, ex))
        ni, nl, nc = ni + len(pi), nl + len(pl), nc + len(pi & pl)
    p = nc / ni if ni else 0.0
    r = nc / nl if nl else 0.0
    f1 = 2 * p * r / (p + r) if nc else 0.0
    f = lambda v, d=torch.float32: W(torch.tensor([v], dtype=d, device=dev()))  # noqa: E731
    return f(p), f(r), f(f1), f(ni, torch.int64), f(nl, torch.int64), f(nc, torch.int64)


def cos_sim(X, Y):
    """row-wise cosine similarity [N, 1]; Y may have a single row (cos_sim_op.h)"""
    x, y = T(X), T(Y)
    x2 = x.reshape(x.shape[0], -1)
    y2 = y.reshape(y.shape[0], -1)
    num = (x2 * y2).sum(1)
    den = x2.norm(dim=1) * y2.norm(dim=1)
    return W((num / den)[:, None])


# ----------------------------------------------------------------------------- activations
def softmax(input, use_cudnn=True, name=None, axis=-1):
    return W(torch.softmax(T(input), axis))


def relu(x, name=None):
    return W(torch.relu(T(x)), x)


def selu(x, scale=None, alpha=None, name=None):
    s = 1.0507009873554804934193349852946 if scale is None else scale
    a = 1.6732632423543772848170429916717 if alpha is None else alpha
    t = T(x)
    return W(s * torch.where(t > 0, t, a * (torch.exp(t) - 1)))


def log(x, name=None):
    return W(torch.log(T(x)), x)


def elu(x, alpha=1.0, name=None):
    return W(TF.elu(T(x), alpha))


def relu6(x, threshold=6.0, name=None):
    return W(T(x).clamp(0, threshold))


def pow(x, factor=1.0, name=None):
    return W(torch.pow(T(x), T(factor) if isinstance(factor, Tensor) else factor))


def stanh(x, scale_a=0.67, scale_b=1.7159, name=None):
    return W(scale_b * torch.tanh(scale_a * T(x)))


def hard_sigmoid(x, slope=0.2, offset=0.5, name=None):
    return W((slope * T(x) + offset).clamp(0, 1))


def swish(x, beta=1.0, name=None):
    t = T(x)
    return W(t * torch.sigmoid(beta * t))


def brelu(x, t_min=0.0, t_max=24.0, name=None):
    return W(T(x).clamp(t_min, t_max))


def leaky_relu(x, alpha=0.02, name=None):
    return W(TF.leaky_relu(T(x), alpha))


def soft_relu(x, threshold=40.0, name=None):
    return W(torch.log1p(torch.exp(T(x).clamp(-threshold, threshold))))


def hard_swish(x, threshold=6.0, scale=6.0, offset=3.0, name=None):
    t = T(x)
    return W(t * (t + offset).clamp(0, threshold) / scale)


def mish(x, threshold=20, name=None):
    t = T(x)
    sp = torch.where(t > threshold, t, torch.where(t < -threshold, torch.exp(t), torch.log1p(torch.exp(t))))
    return W(t * torch.tanh(sp))


def sign(x):
    return W(torch.sign(T(x)))


# ----------------------------------------------------------------------------- pooling
def _pool_pad(pool_padding, nd):
    if isinstance(pool_padding, str):
        return pool_padding.upper()
    p = pool_padding if isinstance(pool_padding, (list, tuple)) else [pool_padding] * nd
    p = [int(v) for v in p]
    if len(p) == nd:
        return [(v, v) for v in p]
    if len(p) == 2 * nd:
        return [(p[2 * i], p[2 * i + 1]) for i in range(nd)]
    raise ValueError(f"pool padding {pool_padding!r}")


def _pool(input, pool_size, pool_type, pool_stride, pool_padding, global_pooling, ceil_mode, exclusive,
          data_format, nd):
    x = T(input)
    cl = data_format[-1] == "C"
    if cl:
        x = x.movedim(-1, 1)
    spatial = list(x.shape[2:])
    if global_pooling:
        y = x.amax(dim=tuple(range(2, 2 + nd)), keepdim=True) if pool_type == "max" else \
            x.mean(dim=tuple(range(2, 2 + nd)), keepdim=True)
        return W(y.movedim(1, -1) if cl else y)
    k = pool_size if isinstance(pool_size, (list, tuple)) else [pool_size] * nd
    s = pool_stride if isinstance(pool_stride, (list, tuple)) else [pool_stride] * nd
    k, s = [int(v) for v in k], [int(v) for v in s]
    pad = _pool_pad(pool_padding, nd)
    if pad == "VALID":
        pad = [(0, 0)] * nd
    elif pad == "SAME":
        pad = []
        for i in range(nd):
            out = -(-spatial[i] // s[i])
            tot = max((out - 1) * s[i] + k[i] - spatial[i], 0)
            pad.append((tot // 2, tot - tot // 2))
    # explicit (possibly asymmetric) padding, then an unpadded pool; ceil_mode adds the tail
    ext = []
    for i in range(nd):
        lo, hi = pad[i]
        if ceil_mode:
            n = spatial[i] + lo + hi
            out = -(-(n - k[i]) // s[i]) + 1
            hi += max((out - 1) * s[i] + k[i] - n, 0)
        ext.append((lo, hi))
    flat = []
    for lo, hi in reversed(ext):
        flat += [lo, hi]
    if pool_type == "max":
        xp = TF.pad(x, flat, value=float("-inf")) if any(flat) else x
        y = [TF.max_pool1d, TF.max_pool2d, TF.max_pool3d][nd - 1](xp, k, s)
    else:
        xp = TF.pad(x, flat) if any(flat) else x
        y = [TF.avg_pool1d, TF.avg_pool2d, TF.avg_pool3d][nd - 1](xp, k, s)
        if exclusive and any(flat):
            ones = TF.pad(torch.ones([1, 1] + spatial, device=x.device, dtype=x.dtype), flat)
            cnt = [TF.avg_pool1d, TF.avg_pool2d, TF.avg_pool3d][nd - 1](ones, k, s)
            y = y / cnt
    return W(y.movedim(1, -1) if cl else y)


def pool2d(input, pool_size=-1, pool_type="max", pool_stride=1, pool_padding=0, global_pooling=False,
           use_cudnn=True, ceil_mode=False, name=None, exclusive=True, data_format="NCHW"):
    return _pool(input, pool_size, pool_type, pool_stride, pool_padding, global_pooling or pool_size == -1,
                 ceil_mode, exclusive, data_format, 2)


def pool3d(input, pool_size=-1, pool_type="max", pool_stride=1, pool_padding=0, global_pooling=False,
           use_cudnn=True, ceil_mode=False, name=None, exclusive=True, data_format="NCDHW"):
    return _pool(input, pool_size, pool_type, pool_stride, pool_padding, global_pooling or pool_size == -1,
                 ceil_mode, exclusive, data_format, 3)


def adaptive_pool2d(input, pool_size, pool_type="max", require_index=False, name=None):
    x = T(input)
    if pool_type == "max":
        y, idx = TF.adaptive_max_pool2d(x, pool_size, return_indices=True)
        return (W(y), W(idx)) if require_index else W(y)
    return W(TF.adaptive_avg_pool2d(x, pool_size))


def adaptive_pool3d(input, pool_size, pool_type="max", require_index=False, name=None):
    x = T(input)
    if pool_type == "max":
        y, idx = TF.adaptive_max_pool3d(x, pool_size, return_indices=True)
        return (W(y), W(idx)) if require_index else W(y)
    return W(TF.adaptive_avg_pool3d(x, pool_size))


# ----------------------------------------------------------------------------- reductions
def _reduce(fn, input, dim, keep_dim):
    x = T(input)
    if x.dim() == 0:
        return W(x)
    axes = norm_axes(dim, x.dim())
    return W(fn(x, axes, keep_dim))


def reduce_sum(input, dim=None, keep_dim=False, name=None):
    return _reduce(lambda x, a, k: x.sum(dim=a, keepdim=k), input, dim, keep_dim)


def reduce_mean(input, dim=None, keep_dim=False, name=None):
    return _reduce(lambda x, a, k: x.mean(dim=a, keepdim=k), input, dim, keep_dim)


def reduce_max(input, dim=None, keep_dim=False, name=None):
    return _reduce(lambda x, a, k: x.amax(dim=a, keepdim=k), input, dim, keep_dim)


def reduce_min(input, dim=None, keep_dim=False, name=None):
    return _reduce(lambda x, a, k: x.amin(dim=a, keepdim=k), input, dim, keep_dim)


def _prod(x, a, k):
    for d in sorted(a, reverse=True):
        x = x.prod(dim=d, keepdim=k)
    return x


def reduce_prod(input, dim=None, keep_dim=False, name=None):
    return _reduce(_prod, input, dim, keep_dim)


def reduce_all(input, dim=None, keep_dim=False, name=None):
    return _reduce(lambda x, a, k: x.bool().all(dim=tuple(a), keepdim=k) if a else x.bool(), input, dim, keep_dim)


def reduce_any(input, dim=None, keep_dim=False, name=None):
    return _reduce(lambda x, a, k: x.bool().any(dim=tuple(a), keepdim=k) if a else x.bool(), input, dim, keep_dim)


def mean(x, name=None):
    return W(T(x).mean())


# ----------------------------------------------------------------------------- dropout / split / misc
def dropout(x, dropout_prob, is_test=None, seed=None, name=None, dropout_implementation="downgrade_in_infer"):
    """downgrade_in_infer: train y = x * mask, infer y = x * (1 - p); upscale_in_train: train
    y = x * mask / (1 - p), infer y = x"""
    t = T(x)
    train = not is_test if is_test is not None else True
    p = float(dropout_prob)
    if not train:
        return W(t * (1.0 - p) if dropout_implementation == "downgrade_in_infer" else t)
    if p >= 1.0:
        return W(torch.zeros_like(t))
    gen = None
    if seed:
        gen = torch.Generator(device=t.device)
        gen.manual_seed(int(seed))
    keep = (torch.rand(t.shape, device=t.device, generator=gen) >= p).to(t.dtype)
    y = t * keep
    if dropout_implementation == "upscale_in_train":
        y = y / (1.0 - p)
    return W(y)


def split(input, num_or_sections, dim=-1, name=None):
    x = T(input)
    d = dim % x.dim()
    if isinstance(num_or_sections, int):
        return [W(p) for p in torch.chunk(x, num_or_sections, d)]
    secs = [int(T(s).item()) if isinstance(s, Tensor) else int(s) for s in num_or_sections]
    if -1 in secs:
        secs[secs.index(-1)] = x.shape[d] - (sum(secs) + 1)
    return [W(p) for p in torch.split(x, secs, d)]


def ctc_greedy_decoder(input, blank, input_length=None, padding_value=0, name=None):
    """argmax per step, merge repeats, drop blanks. LoD input -> LoD output; padded input with
    ``input_length`` -> (padded output, output lengths [N, 1])"""
    x, lens, lod = to_padded(input, input_length)
    ids = x.argmax(-1)
    B, Tm = ids.shape
    outs, out_lens = [], []
    for b in range(B):
        n = int(lens[b])
        seq, prev = [], None
        for t in range(n):
            k = int(ids[b, t])
            if k != prev and k != blank:
                seq.append(k)
            prev = k
        outs.append(seq)
        out_lens.append(len(seq))
    if lod:
        flat = torch.tensor([k for s in outs for k in s] or [], dtype=torch.long, device=x.device).reshape(-1, 1)
        o = W(flat)
        o._lod = [fcore._offsets_from_lengths(out_lens)]
        return o
    Tm2 = max(out_lens + [1])
    out = torch.full((B, Tm2), padding_value, dtype=torch.long, device=x.device)
    for b, s in enumerate(outs):
        if s:
            out[b, :len(s)] = torch.tensor(s, device=x.device)
    return W(out), W(torch.tensor(out_lens, dtype=torch.long, device=x.device)[:, None])


def l2_normalize(x, axis, epsilon=1e-12, name=None):
    t = T(x)
    n = (t * t).sum(axis, keepdim=True).clamp_min(epsilon).sqrt()
    return W(t / n)


def matmul(x, y, transpose_x=False, transpose_y=False, alpha=1.0, name=None):
    a, b = T(x), T(y)
    if transpose_x:
        a = a.transpose(-1, -2) if a.dim() > 1 else a
    if transpose_y:
        b = b.transpose(-1, -2) if b.dim() > 1 else b
    out = torch.matmul(a, b)
    return W(out * alpha if alpha != 1.0 else out)


def topk(input, k, name=None):
    kk = int(T(k).item()) if isinstance(k, Tensor) else int(k)
    v, i = torch.topk(T(input), kk, dim=-1)
    return W(v), W(i)


def transpose(x, perm, name=None):
    return W(T(x).permute(*perm))


def im2sequence(input, filter_size=1, stride=1, padding=0, input_image_size=None, out_stride=1, name=None):
    """[N, C, H, W] -> LoD [N * oh * ow, C * kh * kw], one sequence per image (im2sequence_op.h)"""
    x = T(input)
    k = filter_size if isinstance(filter_size, (list, tuple)) else [filter_size] * 2
    s = stride if isinstance(stride, (list, tuple)) else [stride] * 2
    p = padding if isinstance(padding, (list, tuple)) else [padding] * 4
    if len(p) == 2:
        p = [p[0], p[1], p[0], p[1]]
    xp = TF.pad(x, [p[1], p[3], p[0], p[2]])   # up, left, down, right
    cols = TF.unfold(xp, k, stride=s)           # [N, C*kh*kw, L]
    N, _, L = cols.shape
    out = W(cols.transpose(1, 2).reshape(N * L, -1))
    out._lod = [[i * L for i in range(N + 1)]]
    return out


def multiplex(inputs, index, name=None):
    xs = torch.stack([T(i) for i in inputs], 0)
    idx = T(index).reshape(-1).long()
    return W(xs[idx, torch.arange(idx.shape[0], device=idx.device)])


def smooth_l1(x, y, inside_weight=None, outside_weight=None, sigma=None):
    s2 = (sigma if sigma is not None else 1.0) ** 2
    d = T(x) - T(y)
    if inside_weight is not None:
        d = d * T(inside_weight)
    a = d.abs()
    v = torch.where(a < 1.0 / s2, 0.5 * d * d * s2, a - 0.5 / s2)
    if outside_weight is not None:
        v = v * T(outside_weight)
    return W(v.reshape(v.shape[0], -1).sum(1, keepdim=True))


def one_hot(input, depth, allow_out_of_range=False):
    """one_hot (v1): ``input`` [..., 1] -> [..., depth]"""
    ids = T(input).long()
    if ids.dim() > 1 and ids.shape[-1] == 1:
        ids = ids.squeeze(-1)
    d = int(T(depth).item()) if isinstance(depth, Tensor) else int(depth)
    valid = (ids >= 0) & (ids < d)
    if not allow_out_of_range and not bool(valid.all()):
        raise ValueError("one_hot: index out of range [0, depth)")
    out = TF.one_hot(ids.clamp(0, d - 1), d).float() * valid[..., None].float()
    return W(out)


_step_counters = {}


def autoincreased_step_counter(counter_name=None, begin=1, step=1):
    """persistable int64 counter advanced by ``step`` every time the program (or the call, in
    dygraph) runs; first value is ``begin``"""
    from ...static.program import OpDesc, default_main_program
    name = counter_name or "@STEP_COUNTER@"
    st = _step_counters.setdefault(name, {"v": begin - step})
    if fcore_static():
        from ._common import static_op

        def _tick():
            st["v"] += step
            return W(torch.tensor([st["v"]], dtype=torch.long, device=dev()))
        from ...static.program import Variable
        blk = default_main_program().current_block()
        v = Variable(blk, torch.empty([1], dtype=torch.long, device="meta"), name)
        blk.vars[name] = v
        op = OpDesc("increment", lambda: _tick(), (), {}, v, attrs={"step": float(step)})
        v.op = op
        blk.append_op(op)
        _ = static_op
        return v
    st["v"] += step
    return W(torch.tensor([st["v"]], dtype=torch.long, device=dev()))


def fcore_static():
    from ._common import static_mode
    return static_mode()


def reshape(x, shape, actual_shape=None, act=None, inplace=False, name=None):
    t = T(x)
    if actual_shape is not None:
        shape = [int(v) for v in T(actual_shape).tolist()]
    shp = [int(T(s).item()) if isinstance(s, Tensor) else int(s) for s in
           (T(shape).tolist() if isinstance(shape, Tensor) else shape)]
    shp = [t.shape[i] if v == 0 else v for i, v in enumerate(shp)]
    return act_(W(t.reshape(shp), x), act)


def squeeze(input, axes, name=None):
    t = T(input)
    axes = [a % t.dim() for a in axes] if axes else [i for i, s in enumerate(t.shape) if s == 1]
    keep = [s for i, s in enumerate(t.shape) if not (i in axes and s == 1)]
    return W(t.reshape(keep))


def unsqueeze(input, axes, name=None):
    t = T(input)
    axes = [axes] if isinstance(axes, int) else list(axes)
    for a in axes:
        a = int(T(a).item()) if isinstance(a, Tensor) else a
        t = t.unsqueeze(a if a >= 0 else a + t.dim() + 1)
    return W(t)


def lod_reset(x, y=None, target_lod=None):
    """new LoD from ``y``'s LoD (or its data as offsets) or from ``target_lod`` offsets"""
    out = W(T(x))
    if y is not None:
        ylod = fcore.lod_of(y)
        out._lod = ylod if ylod else [[int(v) for v in T(y).reshape(-1).tolist()]]
    elif target_lod is not None:
        out._lod = [list(map(int, target_lod))]
    else:
        raise ValueError("lod_reset needs y or target_lod")
    return out


def lod_append(x, level):
    out = W(T(x))
    lvl = fcore.lod_of(level) or [[int(v) for v in (T(level).reshape(-1).tolist() if isinstance(level, Tensor)
                                                     else level)]]
    out._lod = fcore.lod_of(x) + [lvl[-1]]
    return out


def lrn(input, n=5, k=1.0, alpha=1e-4, beta=0.75, name=None, data_format="NCHW"):
    """out = x / (k + alpha * sum_{|c'-c| <= n/2} x_{c'}^2) ^ beta  (lrn_op.cc: alpha is NOT
    divided by n)"""
    x = T(input)
    if data_format == "NHWC":
        x = x.permute(0, 3, 1, 2)
    sq = (x * x).unsqueeze(1)
    half = n // 2
    sq = TF.pad(sq, (0, 0, 0, 0, half, n - 1 - half))
    acc = TF.avg_pool3d(sq, (n, 1, 1), stride=1).squeeze(1) * n
    y = x / (k + alpha * acc).pow(beta)
    return W(y.permute(0, 2, 3, 1) if data_format == "NHWC" else y)


def pad(x, paddings, pad_value=0.0, name=None):
    t = T(x)
    flat = []
    for i in reversed(range(t.dim())):
        flat += [int(paddings[2 * i]), int(paddings[2 * i + 1])]
    return W(TF.pad(t, flat, value=pad_value))


def pad_constant_like(x, y, pad_value=0.0, name=None):
    a, b = T(x), T(y)
    flat = []
    for i in reversed(range(b.dim())):
        flat += [0, a.shape[i] - b.shape[i]]
    return W(TF.pad(b, flat, value=pad_value))


def label_smooth(label, prior_dist=None, epsilon=0.1, dtype="float32", name=None):
    return F.label_smooth(label, prior_dist, epsilon)


def roi_pool(input, rois, pooled_height=1, pooled_width=1, spatial_scale=1.0, rois_num=None, name=None):
    from ...vision import ops as V
    return V.roi_pool(input, rois, _rois_num(rois, rois_num), (pooled_height, pooled_width), spatial_scale)


def _rois_num(rois, rois_num):
    if rois_num is not None:
        return rois_num
    off = fcore.lod_of(rois)
    if off:
        return W(torch.tensor(fcore._lengths_from_offsets(off[-1]), dtype=torch.int32, device=dev()))
    return W(torch.tensor([T(rois).shape[0]], dtype=torch.int32, device=dev()))


def roi_align(input, rois, pooled_height=1, pooled_width=1, spatial_scale=1.0, sampling_ratio=-1, rois_num=None,
              name=None, aligned=False):
    from ...vision import ops as V
    return V.roi_align(input, rois, _rois_num(rois, rois_num), (pooled_height, pooled_width), spatial_scale,
                       sampling_ratio, aligned)


def psroi_pool(input, rois, output_channels, spatial_scale, pooled_height, pooled_width, rois_num=None, name=None):
    from ...vision import ops as V
    return V.psroi_pool(input, rois, _rois_num(rois, rois_num), (pooled_height, pooled_width), spatial_scale)


def prroi_pool(input, rois, spatial_scale=1.0, pooled_height=1, pooled_width=1, batch_roi_nums=None, name=None):
    """precise RoI pooling: the exact integral of the bilinear interpolant over each bin divided
    by the bin area (prroi_pool_op.h)"""
    x = T(input)
    r = T(rois).float()
    num = T(_rois_num(rois, batch_roi_nums)).reshape(-1).tolist()
    bidx = torch.repeat_interleave(torch.arange(len(num), device=x.device), torch.tensor(num, device=x.device))
    N, C, H, Wd = x.shape
    out = x.new_zeros(r.shape[0], C, pooled_height, pooled_width)

    def seg(lo, hi, n):
        """[(cell, w_left, w_right)]: integrals of the two hat functions of cell [i, i+1] over
        [lo, hi] ∩ [i, i+1]"""
        res = []
        for i in range(max(int(math.floor(lo)), -1), min(int(math.ceil(hi)), n)):
            a, b = max(lo, i), min(hi, i + 1)
            if b <= a:
                continue
            u0, u1 = a - i, b - i
            wr = (u1 * u1 - u0 * u0) / 2
            res.append((i, (u1 - u0) - wr, wr))
        return res

    def px(b, yy, xx):
        if 0 <= yy < H and 0 <= xx < Wd:
            return x[b, :, yy, xx]
        return x.new_zeros(C)

    for k in range(r.shape[0]):
        b = int(bidx[k])
        x1, y1, x2, y2 = [float(v) * spatial_scale for v in r[k].tolist()]
        bw = max(x2 - x1, 0.0) / pooled_width
        bh = max(y2 - y1, 0.0) / pooled_height
        for ph in range(pooled_height):
            for pw in range(pooled_width):
                hs, he = y1 + ph * bh, y1 + (ph + 1) * bh
                ws, we = x1 + pw * bw, x1 + (pw + 1) * bw
                area = (he - hs) * (we - ws)
                if area <= 0:
                    continue
                acc = x.new_zeros(C)
                for (iy, ay0, ay1) in seg(hs, he, H):
                    for (ix, ax0, ax1) in seg(ws, we, Wd):
                        acc = acc + px(b, iy, ix) * ay0 * ax0 + px(b, iy, ix + 1) * ay0 * ax1 + \
                            px(b, iy + 1, ix) * ay1 * ax0 + px(b, iy + 1, ix + 1) * ay1 * ax1
                out[k, :, ph, pw] = acc / area
    return W(out)


def dice_loss(input, label, epsilon=0.00001, name=None):
    return F.dice_loss(input, label, epsilon)


# ----------------------------------------------------------------------------- resize
def image_resize(input, out_shape=None, scale=None, name=None, resample="BILINEAR", actual_shape=None,
                 align_corners=True, align_mode=1, data_format="NCHW"):
    mode = {"LINEAR": "linear", "BILINEAR": "bilinear", "TRILINEAR": "trilinear", "NEAREST": "nearest",
            "BICUBIC": "bicubic"}[resample.upper()]
    if actual_shape is not None:
        out_shape = [int(v) for v in T(actual_shape).tolist()]
    if isinstance(out_shape, Tensor):
        out_shape = [int(v) for v in T(out_shape).tolist()]
    elif out_shape is not None:
        out_shape = [int(T(v).item()) if isinstance(v, Tensor) else int(v) for v in out_shape]
    if isinstance(scale, Tensor):
        scale = float(T(scale).item())
    return F.interpolate(input, size=out_shape, scale_factor=None if out_shape else scale, mode=mode,
                         align_corners=align_corners if mode != "nearest" else align_corners, align_mode=align_mode,
                         data_format=data_format)


def resize_linear(input, out_shape=None, scale=None, name=None, actual_shape=None, align_corners=True,
                  align_mode=1, data_format="NCW"):
    return image_resize(input, out_shape, scale, name, "LINEAR", actual_shape, align_corners, align_mode, data_format)


def resize_bilinear(input, out_shape=None, scale=None, name=None, actual_shape=None, align_corners=True,
                    align_mode=1, data_format="NCHW"):
    return image_resize(input, out_shape, scale, name, "BILINEAR", actual_shape, align_corners, align_mode,
                        data_format)


def resize_trilinear(input, out_shape=None, scale=None, name=None, actual_shape=None, align_corners=True,
                     align_mode=1, data_format="NCDHW"):
    return image_resize(input, out_shape, scale, name, "TRILINEAR", actual_shape, align_corners, align_mode,
                        data_format)


def resize_nearest(input, out_shape=None, scale=None, name=None, actual_shape=None, align_corners=True,
                   data_format="NCHW"):
    return image_resize(input, out_shape, scale, name, "NEAREST", actual_shape, align_corners, 1, data_format)


def image_resize_short(input, out_short_len, resample="BILINEAR"):
    h, w = T(input).shape[2], T(input).shape[3]
    short, long_ = (h, w) if h < w else (w, h)
    new_long = int(long_ * float(out_short_len) / short + 0.5)
    shape = [out_short_len, new_long] if h < w else [new_long, out_short_len]
    return image_resize(input, out_shape=shape, resample=resample)


# ----------------------------------------------------------------------------- gather / scatter
def gather(input, index, overwrite=True):
    return W(T(input)[T(index).reshape(-1).long()])


def gather_nd(input, index, name=None):
    x, idx = T(input), T(index).long()
    k = idx.shape[-1]
    flat = idx.reshape(-1, k)
    out = x[tuple(flat[:, i] for i in range(k))]
    return W(out.reshape(list(idx.shape[:-1]) + list(x.shape[k:])))


def scatter(input, index, updates, name=None, overwrite=True):
    x = T(input).clone()
    idx = T(index).reshape(-1).long()
    u = T(updates)
    if overwrite:
        x[idx] = u
    else:
        x[idx] = 0
        x = x.index_add(0, idx, u)
    return W(x)


def scatter_nd_add(ref, index, updates, name=None):
    x = T(ref)
    idx = T(index).long()
    k = idx.shape[-1]
    flat = idx.reshape(-1, k)
    u = T(updates).reshape([flat.shape[0]] + list(x.shape[k:]))
    strides = torch.tensor([int(np.prod(x.shape[i + 1:k])) for i in range(k)], device=x.device)
    lin = (flat * strides).sum(1)
    out = x.reshape([-1] + list(x.shape[k:])).index_add(0, lin, u)
    return W(out.reshape(x.shape))


def scatter_nd(index, updates, shape, name=None):
    u = T(updates)
    z = W(torch.zeros([int(s) for s in shape], dtype=u.dtype, device=u.device))
    return scatter_nd_add(z, index, updates)


def random_crop(x, shape, seed=None):
    t = T(x)
    k = len(shape)
    lead = t.shape[:t.dim() - k]
    g = torch.Generator()
    g.manual_seed(int(seed) if isinstance(seed, int) else int(np.random.randint(1 << 30)))
    flat = t.reshape([-1] + list(t.shape[t.dim() - k:]))
    outs = []
    for i in range(flat.shape[0]):
        sl = [i]
        for d in range(k):
            m = flat.shape[1 + d] - shape[d]
            o = int(torch.randint(0, m + 1, (1,), generator=g)) if m > 0 else 0
            sl.append(builtins_slice(o, o + shape[d]))
        outs.append(flat[tuple(sl)])
    return W(torch.stack(outs, 0).reshape(list(lead) + list(shape)))


def mean_iou(input, label, num_classes):
    """(mean IoU [1], wrong [C], correct [C]) over integer predictions / labels"""
    p = T(input).reshape(-1).long()
    y = T(label).reshape(-1).long()
    correct = torch.bincount(p[p == y], minlength=num_classes)[:num_classes]
    pc = torch.bincount(p, minlength=num_classes)[:num_classes]
    yc = torch.bincount(y, minlength=num_classes)[:num_classes]
    wrong = pc + yc - 2 * correct
    denom = (wrong + correct).float()
    valid = denom > 0
    iou = torch.where(valid, correct.float() / denom.clamp_min(1), torch.zeros_like(denom))
    m = iou.sum() / valid.sum().clamp_min(1)
    return W(m.reshape(1)), W(wrong.int()), W(correct.int())


def crop(x, shape=None, offsets=None, name=None):
    t = T(x)
    if isinstance(shape, Tensor):
        shape = list(T(shape).shape) if T(shape).dim() == t.dim() else [int(v) for v in T(shape).tolist()]
    elif shape is None:
        shape = list(t.shape)
    offs = [0] * t.dim() if offsets is None else \
        [int(T(o).item()) if isinstance(o, Tensor) else int(o) for o in
         (T(offsets).tolist() if isinstance(offsets, Tensor) else offsets)]
    sl = tuple(builtins_slice(o, o + (t.shape[i] - o if s == -1 else s)) for i, (o, s) in enumerate(zip(offs, shape)))
    return W(t[sl])


def crop_tensor(x, shape=None, offsets=None, name=None):
    if isinstance(shape, Tensor):
        shape = [int(v) for v in T(shape).tolist()]
    elif shape is not None:
        shape = [int(T(v).item()) if isinstance(v, Tensor) else int(v) for v in shape]
    return crop(x, shape, offsets)


# ----------------------------------------------------------------------------- shape manipulation
def flatten(x, axis=1, name=None):
    t = T(x)
    a = int(np.prod(t.shape[:axis])) if axis > 0 else 1
    return W(t.reshape(a, -1))


def stack(x, axis=0, name=None):
    xs = x if isinstance(x, (list, tuple)) else [x]
    return W(torch.stack([T(v) for v in xs], axis))


def pad2d(input, paddings=[0, 0, 0, 0], mode="constant", pad_value=0.0, data_format="NCHW", name=None):
    t = T(input)
    p = [int(v) for v in (T(paddings).tolist() if isinstance(paddings, Tensor) else paddings)]
    if data_format == "NHWC":
        t = t.permute(0, 3, 1, 2)
    m = {"constant": "constant", "reflect": "reflect", "edge": "replicate"}[mode]
    y = TF.pad(t, [p[2], p[3], p[0], p[1]], mode=m, value=pad_value) if m == "constant" else \
        TF.pad(t, [p[2], p[3], p[0], p[1]], mode=m)
    return W(y.permute(0, 2, 3, 1) if data_format == "NHWC" else y)


def unstack(x, axis=0, num=None):
    return [W(v) for v in torch.unbind(T(x), axis)]


def unbind(input, axis=0):
    return [W(v) for v in torch.unbind(T(input), axis)]


def _unique_first(x):
    flat = T(x).reshape(-1)
    vals = flat.tolist()
    pos, uniq, inv = {}, [], []
    counts = []
    for v in vals:
        if v not in pos:
            pos[v] = len(uniq)
            uniq.append(v)
            counts.append(0)
        inv.append(pos[v])
        counts[pos[v]] += 1
    return flat, uniq, inv, counts


def unique(x, dtype="int32"):
    """(unique values in first-occurrence order, index of each element into them)"""
    flat, uniq, inv, _ = _unique_first(x)
    d = dt(dtype)
    return W(torch.tensor(uniq, dtype=flat.dtype, device=flat.device)), \
        W(torch.tensor(inv, dtype=d, device=flat.device))


def unique_with_counts(x, dtype="int32"):
    flat, uniq, inv, counts = _unique_first(x)
    d = dt(dtype)
    return W(torch.tensor(uniq, dtype=flat.dtype, device=flat.device)), \
        W(torch.tensor(inv, dtype=d, device=flat.device)), W(torch.tensor(counts, dtype=d, device=flat.device))


def expand(x, expand_times, name=None):
    times = [int(T(v).item()) if isinstance(v, Tensor) else int(v) for v in
             (T(expand_times).tolist() if isinstance(expand_times, Tensor) else expand_times)]
    return W(T(x).repeat(*times))


def expand_as(x, target_tensor, name=None):
    t, g = T(x), T(target_tensor)
    return W(t.repeat(*[a // b for a, b in zip(g.shape, t.shape)]))


def scale(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    t = T(x)
    s = T(scale) if isinstance(scale, Tensor) else scale
    y = t * s + bias if bias_after_scale else (t + bias) * s
    return act_(W(y.to(t.dtype) if y.dtype != t.dtype and not t.is_floating_point() else y, x), act)


# ----------------------------------------------------------------------------- elementwise
def _ew(fn):
    def op(x, y, axis=-1, act=None, name=None):
        xt = T(x)
        yt = T(y) if isinstance(y, (Tensor, torch.Tensor)) else torch.as_tensor(y, dtype=xt.dtype, device=xt.device)
        return act_(W(fn(xt, bcast_y(xt, yt, axis)), x), act)
    return op


elementwise_add = _ew(torch.add)
elementwise_sub = _ew(torch.sub)
elementwise_mul = _ew(torch.mul)
elementwise_div = _ew(lambda a, b: a / b if a.is_floating_point() else torch.div(a, b, rounding_mode="trunc"))
elementwise_max = _ew(torch.maximum)
elementwise_min = _ew(torch.minimum)
elementwise_pow = _ew(torch.pow)
elementwise_mod = _ew(torch.remainder)
elementwise_floordiv = _ew(lambda a, b: torch.div(a, b, rounding_mode="floor"))


def _elementwise_op_name(fn_name):
    return fn_name


# ----------------------------------------------------------------------------- random
def _gen(seed, device):
    if not seed:
        return None
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    return g


def uniform_random_batch_size_like(input, shape, dtype="float32", input_dim_idx=0, output_dim_idx=0, min=-1.0,
                                   max=1.0, seed=0):
    shp = list(shape)
    shp[output_dim_idx] = T(input).shape[input_dim_idx]
    d = dev()
    return W(torch.empty(shp, dtype=dt(dtype), device=d).uniform_(min, max, generator=_gen(seed, d)))


def gaussian_random(shape, mean=0.0, std=1.0, seed=0, dtype="float32", name=None):
    d = dev()
    shp = [int(T(s).item()) if isinstance(s, Tensor) else int(s) for s in
           (T(shape).tolist() if isinstance(shape, Tensor) else shape)]
    return W(torch.empty(shp, dtype=dt(dtype), device=d).normal_(mean, std, generator=_gen(seed, d)))


def gaussian_random_batch_size_like(input, shape, input_dim_idx=0, output_dim_idx=0, mean=0.0, std=1.0, seed=0,
                                    dtype="float32"):
    shp = list(shape)
    shp[output_dim_idx] = T(input).shape[input_dim_idx]
    d = dev()
    return W(torch.empty(shp, dtype=dt(dtype), device=d).normal_(mean, std, generator=_gen(seed, d)))


def uniform_random(shape, dtype="float32", min=-1.0, max=1.0, seed=0, name=None):
    d = dev()
    shp = [int(T(s).item()) if isinstance(s, Tensor) else int(s) for s in
           (T(shape).tolist() if isinstance(shape, Tensor) else shape)]
    return W(torch.empty(shp, dtype=dt(dtype), device=d).uniform_(min, max, generator=_gen(seed, d)))


def sampling_id(x, min=0.0, max=1.0, seed=0, dtype="float32"):
    """one class id per row sampled from the row's (unnormalised, non-negative) distribution"""
    p = T(x).float()
    g = _gen(seed, p.device)
    return W(torch.multinomial(p.clamp_min(0) + 1e-20, 1, generator=g).reshape(-1))


# ----------------------------------------------------------------------------- misc tensor ops
def sum(x):
    xs = x if isinstance(x, (list, tuple)) else [x]
    out = T(xs[0])
    for v in xs[1:]:
        out = out + T(v)
    return W(out)


def slice(input, axes, starts, ends):
    t = T(input)
    sl = [builtins_slice(None)] * t.dim()
    val = lambda v: int(T(v).item()) if isinstance(v, Tensor) else int(v)  # noqa: E731
    if isinstance(starts, Tensor):
        starts = T(starts).tolist()
    if isinstance(ends, Tensor):
        ends = T(ends).tolist()
    for a, s, e in zip(axes, starts, ends):
        n = t.shape[a]
        s, e = val(s), val(e)
        s = max(s + n, 0) if s < 0 else min(s, n)
        e = max(e + n, 0) if e < 0 else min(e, n)
        sl[a] = builtins_slice(s, max(e, s))
    return W(t[tuple(sl)])


def strided_slice(input, axes, starts, ends, strides):
    t = T(input)
    for a, s, e, st in zip(axes, starts, ends, strides):
        n = t.shape[a]
        s, e, st = int(s), int(e), int(st)
        if st > 0:
            s = max(s + n, 0) if s < 0 else min(s, n)
            e = max(e + n, 0) if e < 0 else min(e, n)
            idx = torch.arange(s, e, st, device=t.device)
        else:
            s = s + n if s < 0 else min(s, n - 1)
            e = e + n if e < -1 else (e if e >= 0 else -1)
            idx = torch.arange(s, e, st, device=t.device)
        t = t.index_select(a, idx)
    return W(t)


def shape(input):
    return W(torch.tensor(list(T(input).shape), dtype=torch.int32, device=dev()))


def rank(input):
    return W(torch.tensor(T(input).dim(), dtype=torch.int32, device=dev()))


def size(input):
    return W(torch.tensor([T(input).numel()], dtype=torch.int64, device=dev()))


def _logical(fn, opname):
    def compute(x, y):
        return W(fn(T(x).bool(), T(y).bool()))

    def op(x, y, out=None, name=None):
        from ...framework.dispatch import static_op
        r = static_op(compute, opname)(x, y)
        return write_to(out, r) if out is not None else r
    return op


logical_and = _logical(torch.logical_and, "logical_and")
logical_or = _logical(torch.logical_or, "logical_or")
logical_xor = _logical(torch.logical_xor, "logical_xor")


def _logical_not(x):
    return W(torch.logical_not(T(x).bool()))


def logical_not(x, out=None, name=None):
    from ...framework.dispatch import static_op
    r = static_op(_logical_not, "logical_not")(x)
    return write_to(out, r) if out is not None else r


def clip(x, min, max, name=None):
    return W(T(x).clamp(min, max))


def clip_by_norm(x, max_norm, name=None):
    t = T(x)
    n = t.norm()
    return W(torch.where(n > max_norm, t * (max_norm / n), t))


def mul(x, y, x_num_col_dims=1, y_num_col_dims=1, name=None):
    a, b = T(x), T(y)
    a2 = a.reshape(int(np.prod(a.shape[:x_num_col_dims])), -1)
    b2 = b.reshape(int(np.prod(b.shape[:y_num_col_dims])), -1)
    out = a2 @ b2
    return W(out.reshape(list(a.shape[:x_num_col_dims]) + list(b.shape[y_num_col_dims:])))


def maxout(x, groups, name=None, axis=1):
    t = T(x)
    a = axis % t.dim()
    shp = list(t.shape)
    shp[a:a + 1] = [shp[a] // groups, groups]
    return W(t.reshape(shp).amax(a + 1))


def space_to_depth(x, blocksize, name=None):
    """space_to_depth_op.h index map, reproduced exactly: element (b, k, j, i) of X goes to
    position (b, k % oc, j*bs + (k // oc) // bs, i*bs + (k // oc) % bs) of a [B, oc, H*bs, W*bs]
    image (oc = C / bs^2) whose flat buffer is then read as [B, C*bs^2, H/bs, W/bs]"""
    t = T(x)
    B, C, H, Wd = t.shape
    bs = int(blocksize)
    oc = C // (bs * bs)
    y = t.reshape(B, bs, bs, oc, H, Wd).permute(0, 3, 4, 1, 5, 2).reshape(-1)
    return W(y.reshape(B, C * bs * bs, H // bs, Wd // bs))


def affine_grid(theta, out_shape, name=None):
    if isinstance(out_shape, Tensor):
        out_shape = [int(v) for v in T(out_shape).tolist()]
    return F.affine_grid(theta, out_shape, align_corners=True)


def similarity_focus(input, axis, indexes, name=None):
    """mask of the greedy row/column-exclusive maxima of each selected slice
    (similarity_focus_op.h), broadcast over ``axis``"""
    x = T(input)
    B = x.shape[0]
    out = torch.zeros_like(x)
    xc = x.detach().cpu()
    for b in range(B):
        for idx in indexes:
            sl = xc[b].select(axis - 1, idx)          # 2-D
            r, c = sl.shape
            order = torch.argsort(sl.reshape(-1), descending=True, stable=True).tolist()
            tr, tc, n = [False] * r, [False] * c, 0
            for o in order:
                i, j = o // c, o % c
                if tr[i] or tc[j]:
                    continue
                tr[i] = tc[j] = True
                n += 1
                ix = [b, builtins_slice(None), builtins_slice(None), builtins_slice(None)]
                rest = [d for d in (1, 2, 3) if d != axis]
                ix[rest[0]], ix[rest[1]] = i, j
                out[tuple(ix)] = 1
                if n == min(r, c):
                    break
    return W(out)


def hash(input, hash_size, num_hash=1, name=None):
    """XXH64 of each row's int64 bytes with seeds 0..num_hash-1, mod hash_size ->
    [N, num_hash, 1] (hash_op.h)"""
    import xxhash
    x = T(input).long().cpu().numpy()
    rows = x.reshape(x.shape[0], -1)
    out = np.zeros((rows.shape[0], num_hash, 1), dtype=np.int64)
    for i, row in enumerate(rows):
        buf = np.ascontiguousarray(row).tobytes()
        for j in range(num_hash):
            out[i, j, 0] = xxhash.xxh64_intdigest(buf, seed=j) % hash_size
    return W(torch.from_numpy(out).to(dev()))


def grid_sampler(x, grid, name=None):
    return F.grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=True)


def log_loss(input, label, epsilon=1e-4, name=None):
    return F.log_loss(input, label, epsilon)


def add_position_encoding(input, alpha, beta, name=None):
    """out = alpha * x + beta * PE, PE[t, k] = sin(t / 10000^(k/(half-1))) for the first half of
    the features and cos(...) for the second (add_position_encoding_op.h)"""
    x, lens, lod = to_padded(input)
    B, Tm, D = x.shape
    half = D // 2
    t = torch.arange(Tm, dtype=torch.float64, device=x.device)[:, None]
    k = torch.arange(half, dtype=torch.float64, device=x.device)[None, :]
    val = t / torch.pow(10000.0, k / (half - 1)) if half > 1 else t / 10000.0
    pe = torch.cat([torch.sin(val), torch.cos(val)], 1).to(x.dtype)
    y = alpha * x + beta * pe[None]
    if lod:
        return from_padded(y, lens, fcore.lod_of(input))
    return W(y)


def merge_selected_rows(x, name=None):
    return W(T(x))


def get_tensor_from_selected_rows(x, name=None):
    return W(T(x))


def shuffle_channel(x, group, name=None):
    t = T(x)
    B, C, H, Wd = t.shape
    return W(t.reshape(B, group, C // group, H, Wd).transpose(1, 2).reshape(B, C, H, Wd))


def temporal_shift(x, seg_num, shift_ratio=0.25, name=None, data_format="NCHW"):
    return F.temporal_shift(x, seg_num, shift_ratio, data_format=data_format)


def pixel_shuffle(x, upscale_factor):
    return W(TF.pixel_shuffle(T(x), upscale_factor))


def fsp_matrix(x, y):
    a, b = T(x), T(y)
    B, C1, H, Wd = a.shape
    return W(torch.bmm(a.reshape(B, C1, -1), b.reshape(B, b.shape[1], -1).transpose(1, 2)) / (H * Wd))


def continuous_value_model(input, cvm, use_cvm=True):
    x = T(input)
    if not use_cvm:
        return W(x[:, 2:])
    show = torch.log(x[:, 0:1] + 1)
    click = torch.log(x[:, 1:2] + 1) - show
    return W(torch.cat([show, click, x[:, 2:]], 1))


def where(condition):
    return W(torch.nonzero(T(condition).bool()).long())


def unfold(x, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    return F.unfold(x, kernel_sizes, strides, paddings, dilations)


def deformable_roi_pooling(input, rois, trans, no_trans=False, spatial_scale=1.0, group_size=[1, 1],
                           pooled_height=1, pooled_width=1, part_size=None, sample_per_part=1, trans_std=0.1,
                           position_sensitive=False, name=None):
    """deformable (position-sensitive) RoI pooling (deformable_psroi_pooling_op.h): each bin is
    shifted by trans * trans_std * roi size and averaged over sample_per_part^2 bilinear samples"""
    x = T(input)
    r = T(rois).float()
    tr = T(trans) if not no_trans else None
    N, C, H, Wd = x.shape
    ph_, pw_ = pooled_height, pooled_width
    part = part_size or [ph_, pw_]
    gh, gw = group_size
    oc = C // (gh * gw) if position_sensitive else C
    num = T(_rois_num(rois, None)).reshape(-1).tolist()
    bidx = torch.repeat_interleave(torch.arange(len(num)), torch.tensor(num)).tolist()
    out = x.new_zeros(r.shape[0], oc, ph_, pw_)

    def bil(b, c, yy, xx):
        if yy < -0.5 or yy > H - 0.5 or xx < -0.5 or xx > Wd - 0.5:
            return None
        yy, xx = min(max(yy, 0.0), H - 1.0), min(max(xx, 0.0), Wd - 1.0)
        y0, x0 = int(math.floor(yy)), int(math.floor(xx))
        y1, x1 = min(y0 + 1, H - 1), min(x0 + 1, Wd - 1)
        ly, lx = yy - y0, xx - x0
        return (x[b, c, y0, x0] * (1 - ly) * (1 - lx) + x[b, c, y0, x1] * (1 - ly) * lx +
                x[b, c, y1, x0] * ly * (1 - lx) + x[b, c, y1, x1] * ly * lx)

    for k in range(r.shape[0]):
        b = bidx[k]
        x1 = round(float(r[k, 0])) * spatial_scale - 0.5
        y1 = round(float(r[k, 1])) * spatial_scale - 0.5
        x2 = (round(float(r[k, 2])) + 1.0) * spatial_scale - 0.5
        y2 = (round(float(r[k, 3])) + 1.0) * spatial_scale - 0.5
        rw, rh = max(x2 - x1, 0.1), max(y2 - y1, 0.1)
        bw, bh = rw / pw_, rh / ph_
        sw, sh = bw / sample_per_part, bh / sample_per_part
        for c in range(oc):
            for i in range(ph_):
                for j in range(pw_):
                    pi, pj = int(i * part[0] / ph_), int(j * part[1] / pw_)
                    dx = dy = 0.0
                    if tr is not None:
                        cls = c // max(oc // (tr.shape[1] // 2), 1) if tr.shape[1] > 2 else 0
                        dx = float(tr[k, 2 * cls, pi, pj]) * trans_std
                        dy = float(tr[k, 2 * cls + 1, pi, pj]) * trans_std
                    ws = j * bw + x1 + dx * rw
                    hs = i * bh + y1 + dy * rh
                    gi, gj = min(max(int(i * gh / ph_), 0), gh - 1), min(max(int(j * gw / pw_), 0), gw - 1)
                    cc = (c * gh + gi) * gw + gj if position_sensitive else c
                    acc, cnt = 0.0, 0
                    for ih in range(sample_per_part):
                        for iw in range(sample_per_part):
                            v = bil(b, cc, hs + ih * sh, ws + iw * sw)
                            if v is not None:
                                acc = acc + v
                                cnt += 1
                    out[k, c, i, j] = acc / cnt if cnt else 0.0
    return W(out)


def filter_by_instag(ins, ins_tag, filter_tag, is_lod, out_val_if_empty=0):
    """keep the instances (rows, or LoD sequences when ``is_lod``) whose tag list intersects
    ``filter_tag``; -> (filtered rows, loss weight [n, 1], index map [n, 3])"""
    x = T(ins)
    tags = fcore.lod_of(ins_tag)
    tag_vals = T(ins_tag).reshape(-1).tolist()
    toff = tags[-1] if tags else list(range(len(tag_vals) + 1))
    want = set(int(v) for v in T(filter_tag).reshape(-1).tolist())
    ioff = fcore.lod_of(ins)[-1] if is_lod and fcore.lod_of(ins) else list(range(x.shape[0] + 1))
    keep, imap, pos = [], [], 0
    for i in range(len(ioff) - 1):
        if set(int(v) for v in tag_vals[toff[i]:toff[i + 1]]) & want:
            a, b = ioff[i], ioff[i + 1]
            keep.append(x[a:b])
            imap.append([pos, a, b - a])
            pos += b - a
    if not keep:
        out = torch.full([1] + list(x.shape[1:]), float(out_val_if_empty), dtype=x.dtype, device=x.device)
        return W(out), W(torch.zeros(1, 1, device=x.device)), W(torch.zeros(1, 3, dtype=torch.long))
    out = torch.cat(keep, 0)
    return W(out), W(torch.ones(out.shape[0], 1, device=x.device)), W(torch.tensor(imap, dtype=torch.long))


def shard_index(input, index_num, nshards, shard_id, ignore_value=-1):
    x = T(input).long()
    ss = (index_num + nshards - 1) // nshards
    return W(torch.where(x // ss == shard_id, x - shard_id * ss, torch.full_like(x, ignore_value)))


def gather_tree(ids, parents):
    return F.gather_tree(ids, parents)


register(globals(), __all__, skip=_BUILDERS)
register(globals(), ["_lookup_v1"])   # embedding's recorded op (lookup_table in a saved ProgramDesc)
_ = (dt, Tensor)
