"""``paddle.static.nn`` (reference: python/paddle/static/nn/__init__.py, fluid/layers/nn.py,
control_flow.py, sequence_lod.py). Parameter-creating builders (fc, conv2d, batch_norm …)
create their parameters eagerly in the global scope and emit functional ops (recorded when
called on static Variables). Control flow records one op whose replay evaluates the
predicate and runs the chosen branch. The sequence ops are fluid.layers.sequence_lod's (LoD inputs)."""
from __future__ import annotations

import numpy as np
import torch

from ..framework.core import Tensor, _wrap, convert_dtype
from ..framework.dispatch import register_ops, static_op
from ..framework.param_attr import ParamAttr
from ..nn import functional as F
from ..nn import initializer as I
from ..nn.layer.layers import _create_parameter
from ..utils import unique_name as _unique_name

__all__ = ["fc", "batch_norm", "embedding", "sparse_embedding", "conv2d", "conv2d_transpose", "conv3d",
           "conv3d_transpose", "layer_norm", "group_norm", "instance_norm", "data_norm", "prelu",
           "bilinear_tensor_product", "deform_conv2d", "spectral_norm", "nce", "row_conv", "crf_decoding",
           "multi_box_head", "py_func", "cond", "case", "switch_case", "while_loop", "StaticRNN",
           "sequence_concat", "sequence_conv", "sequence_enumerate", "sequence_expand", "sequence_expand_as",
           "sequence_first_step", "sequence_last_step", "sequence_pad", "sequence_pool", "sequence_reshape",
           "sequence_reverse", "sequence_scatter", "sequence_slice", "sequence_softmax", "sequence_unpad"]


def _act(x, act):
    return getattr(F, act)(x) if act else x


def fc(x, size, num_flatten_dims=1, weight_attr=None, bias_attr=None, activation=None, name=None):
    _h = name or _unique_name.generate("fc")
    xs = x if isinstance(x, (list, tuple)) else [x]
    out = None
    for xi in xs:
        in_dim = int(np.prod(xi.shape[num_flatten_dims:]))
        w = _create_parameter([in_dim, size], xi.dtype, weight_attr, helper=_h)
        from ..tensor import reshape
        flat = reshape(xi, [-1 if num_flatten_dims == 1 else 0] * 0 + list(xi.shape[:num_flatten_dims]) + [in_dim]) \
            if len(xi.shape) != num_flatten_dims + 1 else xi
        y = F.linear(flat, w)
        out = y if out is None else out + y
    if bias_attr is not False:
        b = _create_parameter([size], out.dtype, bias_attr, is_bias=True, helper=_h)
        out = out + b
    return _act(out, activation)


def batch_norm(input, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None, bias_attr=None,
               data_layout="NCHW", in_place=False, name=None, moving_mean_name=None, moving_variance_name=None,
               do_model_average_for_mean_and_var=True, use_global_stats=False):
    _h = name or _unique_name.generate("batch_norm")
    c = input.shape[1] if data_layout == "NCHW" else input.shape[-1]
    w = _create_parameter([c], "float32", param_attr, default_initializer=I.Constant(1.0), helper=_h)
    b = _create_parameter([c], "float32", bias_attr, is_bias=True, helper=_h)
    from ..framework import core
    mean = _wrap(torch.zeros(c, device=core.default_device()))
    var = _wrap(torch.ones(c, device=core.default_device()))
    mean.name = moving_mean_name or (w.name + "_mean")
    var.name = moving_variance_name or (w.name + "_variance")
    y = F.batch_norm(input, mean, var, w, b, training=not is_test, momentum=momentum, epsilon=epsilon,
                     data_format=data_layout, use_global_stats=use_global_stats)
    return _act(y, act)


def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None, param_attr=None, dtype="float32"):
    _h = _unique_name.generate("embedding")
    w = _create_parameter(list(size), dtype, param_attr, default_initializer=I.XavierUniform(), helper=_h)
    return F.embedding(input, w, padding_idx)


def sparse_embedding(input, size, padding_idx=None, is_test=False, entry=None, table_class="MemorySparseTable",
                     param_attr=None, dtype="float32", slot=None):
    """Parameter-server mode (fleet.init with a PS role maker + init_worker): rows live in a
    server sparse table (parallel/ps DistributedEmbedding); otherwise a local embedding."""
    from ..parallel import ps
    if ps._runtime is not None and ps._runtime.client is not None:
        return ps.sparse_embedding(input, size, padding_idx=padding_idx, is_test=is_test, entry=entry,
                                   param_attr=param_attr)
    return embedding(input, size, padding_idx=padding_idx, param_attr=param_attr, dtype=dtype)


def _conv(fn, transpose, input, num_filters, filter_size, stride, padding, dilation, groups, param_attr, bias_attr,
          act, data_format, nd, output_size=None):
    _h = _unique_name.generate(fn.__name__)   # conv2d / conv3d / conv2d_transpose / conv3d_transpose
    cin = input.shape[1] if data_format[1] == "C" else input.shape[-1]
    k = filter_size if isinstance(filter_size, (list, tuple)) else [filter_size] * nd
    shape = ([cin, num_filters // (groups or 1)] if transpose else [num_filters, cin // (groups or 1)]) + list(k)
    fan_in = cin // (groups or 1) * int(np.prod(k))
    w = _create_parameter(shape, input.dtype, param_attr, default_initializer=I.Normal(0.0, (2.0 / fan_in) ** 0.5),
                          helper=_h)
    b = None if bias_attr is False else _create_parameter([num_filters], input.dtype, bias_attr, is_bias=True, helper=_h)
    if transpose:
        y = fn(input, w, b, stride, padding, 0, dilation, groups or 1, output_size, data_format) if nd == 2 else \
            fn(input, w, b, stride, padding, 0, groups or 1, dilation, output_size, data_format)
    else:
        y = fn(input, w, b, stride, padding, dilation, groups or 1, data_format)
    return _act(y, act)


def conv2d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None, param_attr=None,
           bias_attr=None, use_cudnn=True, act=None, name=None, data_format="NCHW"):
    return _conv(F.conv2d, False, input, num_filters, filter_size, stride, padding, dilation, groups, param_attr,
                 bias_attr, act, data_format, 2)


def conv3d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None, param_attr=None,
           bias_attr=None, use_cudnn=True, act=None, name=None, data_format="NCDHW"):
    return _conv(F.conv3d, False, input, num_filters, filter_size, stride, padding, dilation, groups, param_attr,
                 bias_attr, act, data_format, 3)


def conv2d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,
                     groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
                     data_format="NCHW"):
    return _conv(F.conv2d_transpose, True, input, num_filters, filter_size or 3, stride, padding, dilation, groups,
                 param_attr, bias_attr, act, data_format, 2, output_size)


def conv3d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,
                     groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
                     data_format="NCDHW"):
    return _conv(F.conv3d_transpose, True, input, num_filters, filter_size or 3, stride, padding, dilation, groups,
                 param_attr, bias_attr, act, data_format, 3, output_size)


def layer_norm(input, scale=True, shift=True, begin_norm_axis=1, epsilon=1e-05, param_attr=None, bias_attr=None,
               act=None, name=None):
    _h = name or _unique_name.generate("layer_norm")
    shape = input.shape[begin_norm_axis:]
    n = int(np.prod(shape))
    w = _create_parameter([n], "float32", param_attr, default_initializer=I.Constant(1.0), helper=_h) if scale else None
    b = _create_parameter([n], "float32", bias_attr, is_bias=True, helper=_h) if shift else None
    return _act(F.layer_norm(input, shape, w, b, epsilon), act)


def group_norm(input, groups, epsilon=1e-05, param_attr=None, bias_attr=None, act=None, data_layout="NCHW", name=None):
    _h = name or _unique_name.generate("group_norm")
    c = input.shape[1] if data_layout == "NCHW" else input.shape[-1]
    w = _create_parameter([c], "float32", param_attr, default_initializer=I.Constant(1.0), helper=_h)
    b = _create_parameter([c], "float32", bias_attr, is_bias=True, helper=_h)
    return _act(F.group_norm(input, groups, epsilon, w, b, data_layout), act)


def instance_norm(input, epsilon=1e-05, param_attr=None, bias_attr=None, name=None):
    _h = name or _unique_name.generate("instance_norm")
    c = input.shape[1]
    w = _create_parameter([c], "float32", param_attr, default_initializer=I.Constant(1.0), helper=_h)
    b = _create_parameter([c], "float32", bias_attr, is_bias=True, helper=_h)
    return F.instance_norm(input, weight=w, bias=b, eps=epsilon)


def data_norm(input, act=None, epsilon=1e-05, param_attr=None, data_layout="NCHW", in_place=False, name=None,
              moving_mean_name=None, moving_variance_name=None, do_model_average_for_mean_and_var=True,
              slot_dim=-1, sync_stats=False, summary_decay_rate=0.9999999, enable_scale_and_shift=False):
    c = input.shape[-1]
    from ..framework import core
    bsize = _wrap(torch.full([c], 1e4, device=core.default_device()))
    bsum = _wrap(torch.zeros([c], device=core.default_device()))
    bsq = _wrap(torch.full([c], 1e4, device=core.default_device()))

    def _dn(x, n, s, q):
        mean = s._t / n._t
        scale = torch.sqrt(n._t / q._t)
        return _wrap((x._t - mean) * scale)
    return _act(static_op(_dn, "data_norm")(input, bsize, bsum, bsq), act)


def prelu(x, mode, param_attr=None, data_format="NCHW", name=None):
    _h = name or _unique_name.generate("prelu")
    if mode == "all":
        shape = [1]
    elif mode == "channel":
        shape = [x.shape[1] if data_format == "NCHW" else x.shape[-1]]
    else:
        shape = list(x.shape[1:])
    w = _create_parameter(shape, "float32", param_attr, default_initializer=I.Constant(0.25), helper=_h)

    def _prelu(x, w):
        t, wt = x._t, w._t
        if mode == "element":
            return _wrap(torch.where(t > 0, t, t * wt))
        return F.prelu(x, w, data_format)
    return static_op(_prelu, "prelu_static")(x, w)


def bilinear_tensor_product(x, y, size, act=None, name=None, param_attr=None, bias_attr=None):
    _h = name or _unique_name.generate("bilinear_tensor_product")
    w = _create_parameter([size, x.shape[-1], y.shape[-1]], "float32", param_attr, helper=_h)
    b = None if bias_attr is False else _create_parameter([1, size], "float32", bias_attr, is_bias=True, helper=_h)
    return _act(F.bilinear(x, y, w, b), act)


def deform_conv2d(x, offset, mask, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=1,
                  deformable_groups=1, im2col_step=1, weight_attr=None, bias_attr=None, name=None):
    _h = name or _unique_name.generate("deformable_conv")
    from ..vision.ops import deform_conv2d as _dc
    k = filter_size if isinstance(filter_size, (list, tuple)) else [filter_size] * 2
    w = _create_parameter([num_filters, x.shape[1] // groups] + list(k), "float32", weight_attr, helper=_h)
    b = None if bias_attr is False else _create_parameter([num_filters], "float32", bias_attr, is_bias=True, helper=_h)
    return static_op(_dc, "deform_conv2d")(x, offset, w, b, stride, padding, dilation, deformable_groups, groups, mask)


def spectral_norm(weight, dim=0, power_iters=1, eps=1e-12, name=None):
    from ..nn.layer.conv_norm_pool import SpectralNorm
    sn = SpectralNorm(weight.shape, dim, power_iters, eps)
    return static_op(lambda w: sn(w), "spectral_norm")(weight)


def nce(input, label, num_total_classes, sample_weight=None, param_attr=None, bias_attr=None, num_neg_samples=None,
        name=None, sampler="uniform", custom_dist=None, seed=0, is_sparse=False):
    _h = name or _unique_name.generate("nce")
    dim = input.shape[-1]
    w = _create_parameter([num_total_classes, dim], "float32", param_attr, helper=_h)
    b = _create_parameter([num_total_classes, 1], "float32", bias_attr, is_bias=True, helper=_h)
    k = num_neg_samples or 10

    def _nce(x, lab, w, b):
        xt, lt = x._t, lab._t.reshape(-1).long()
        neg = torch.randint(0, num_total_classes, (xt.shape[0], k), device=xt.device)
        pos_logit = (xt * w._t[lt]).sum(-1) + b._t[lt, 0]
        neg_logit = torch.einsum("bd,bkd->bk", xt, w._t[neg]) + b._t[neg, 0]
        pq = k / num_total_classes
        loss = -torch.nn.functional.logsigmoid(pos_logit - np.log(pq)) - \
            torch.nn.functional.logsigmoid(-(neg_logit - np.log(pq))).sum(-1)
        return _wrap(loss.unsqueeze(-1))
    return static_op(_nce, "nce")(input, label, w, b)


def row_conv(input, future_context_size, param_attr=None, act=None):
    _h = _unique_name.generate("row_conv")
    d = input.shape[-1]
    w = _create_parameter([future_context_size + 1, d], "float32", param_attr, helper=_h)

    def _rc(x, w):
        t = x._t
        T = t.shape[1]
        out = torch.zeros_like(t)
        for i in range(future_context_size + 1):
            out[:, :T - i] += t[:, i:] * w._t[i]
        return _wrap(out)
    return _act(static_op(_rc, "row_conv")(input, w), act)


def crf_decoding(input, param_attr, label=None, length=None):
    _h = _unique_name.generate("crf_decoding")
    from ..text import viterbi_decode
    n = input.shape[-1]
    trans = _create_parameter([n + 2, n], "float32", param_attr, helper=_h)

    def _crf(x, tr, ln):
        lens = ln._t if ln is not None else torch.full((x._t.shape[0],), x._t.shape[1], dtype=torch.int64, device=x._t.device)
        _, path = viterbi_decode(x, _wrap(tr._t[2:]), _wrap(lens), include_bos_eos_tag=False)
        return path
    return static_op(_crf, "crf_decoding")(input, trans, length)


def multi_box_head(inputs, image, base_size, num_classes, aspect_ratios, min_ratio=None, max_ratio=None, min_sizes=None,
                   max_sizes=None, steps=None, step_w=None, step_h=None, offset=0.5, variance=[0.1, 0.1, 0.2, 0.2],
                   flip=True, clip=False, kernel_size=1, pad=0, stride=1, name=None, min_max_aspect_ratios_order=False):
    from ..vision.ops import prior_box
    from ..tensor import concat, reshape, transpose
    locs, confs, boxes, vars_ = [], [], [], []
    n = len(inputs)
    if min_sizes is None:
        step = int((max_ratio - min_ratio) / max(n - 2, 1))
        min_sizes, max_sizes = [base_size * 0.1], [base_size * 0.2]
        for r in range(min_ratio, max_ratio + 1, step):
            min_sizes.append(base_size * r / 100.0)
            max_sizes.append(base_size * (r + step) / 100.0)
    for i, x in enumerate(inputs):
        ar = aspect_ratios[i] if isinstance(aspect_ratios[i], (list, tuple)) else [aspect_ratios[i]]
        b, v = prior_box(x, image, [min_sizes[i]], [max_sizes[i]] if max_sizes else None, ar, variance, flip, clip,
                         [step_w[i] if step_w else 0.0, step_h[i] if step_h else 0.0], offset)
        npri = b.shape[2]
        loc = conv2d(x, npri * 4, kernel_size, stride, pad)
        conf = conv2d(x, npri * num_classes, kernel_size, stride, pad)
        locs.append(reshape(transpose(loc, [0, 2, 3, 1]), [0, -1, 4]))
        confs.append(reshape(transpose(conf, [0, 2, 3, 1]), [0, -1, num_classes]))
        boxes.append(reshape(b, [-1, 4]))
        vars_.append(reshape(v, [-1, 4]))
    return concat(locs, 1), concat(confs, 1), concat(boxes, 0), concat(vars_, 0)


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    from . import py_func as _pf
    return _pf(func, x, out, backward_func, skip_vars_in_backward_input)


# ----------------------------------------------------------------------------- control flow
def _truth(p):
    return bool(p._t.reshape(-1)[0].item()) if isinstance(p, Tensor) else bool(p)


def _cond(pred, true_fn, false_fn):
    if _truth(pred):
        return true_fn() if true_fn is not None else None
    return false_fn() if false_fn is not None else None


def cond(pred, true_fn=None, false_fn=None, name=None, return_names=None):
    """dynamic mode / Python predicate: run the taken branch; static Variable predicate: record
    both branches as sub-blocks and one conditional_block op (static/control_flow.py)"""
    from .program import Variable
    if isinstance(pred, Variable):
        from . import control_flow
        return control_flow.cond(pred, true_fn, false_fn)
    return _cond(pred, true_fn, false_fn)


def _case(preds, fns, default):
    for p, f in zip(preds, fns):
        if _truth(p):
            return f()
    return default() if default is not None else None


def case(pred_fn_pairs, default=None, name=None):
    preds = [p for p, _ in pred_fn_pairs]
    fns = [f for _, f in pred_fn_pairs]
    return static_op(_case, "case")(preds, fns, default)


def _switch(index, keys, fns, default):
    i = int(index._t.reshape(-1)[0].item()) if isinstance(index, Tensor) else int(index)
    for k, f in zip(keys, fns):
        if k == i:
            return f()
    return default() if default is not None else fns[-1]()


def switch_case(branch_index, branch_fns, default=None, name=None):
    items = list(branch_fns.items()) if isinstance(branch_fns, dict) else \
        [(i, f) if not isinstance(f, tuple) else f for i, f in enumerate(branch_fns)]
    keys = [k for k, _ in items]
    fns = [f for _, f in items]
    return static_op(_switch, "switch_case")(branch_index, keys, fns, default)


def _while(cond_fn, body, loop_vars):
    vals = list(loop_vars)
    while _truth(cond_fn(*vals)):
        out = body(*vals)
        vals = list(out) if isinstance(out, (list, tuple)) else [out]
    return vals


def while_loop(cond, body, loop_vars, is_test=False, name=None):
    from .program import Variable
    from ..framework import core as _c
    if not _c.in_dynamic_mode() and any(isinstance(v, Variable) for v in loop_vars):
        from . import control_flow
        return control_flow.while_loop(cond, body, loop_vars)
    return _while(cond, body, list(loop_vars))


class StaticRNN:
    """Step-function RNN builder (reference: fluid/layers/control_flow.py:StaticRNN), unrolled
    over the time axis of its step inputs at run time."""

    def __init__(self, name=None):
        self._inputs, self._memories, self._outputs = [], [], []
        self._step_fn = None

    def step(self):
        rnn = self

        class _Ctx:
            def __enter__(self_):
                return rnn

            def __exit__(self_, *a):
                return False
        return _Ctx()

    def step_input(self, x):
        self._inputs.append(x)
        return x

    def memory(self, init=None, shape=None, batch_ref=None, init_value=0.0, init_batch_dim_idx=0, ref_batch_dim_idx=1):
        m = init if init is not None else _wrap(torch.full([batch_ref.shape[ref_batch_dim_idx]] + list(shape[1:]), init_value))
        self._memories.append(m)
        return m

    def update_memory(self, mem, var):
        pass

    def step_output(self, o):
        self._outputs.append(o)

    def output(self, *outputs):
        for o in outputs:
            self.step_output(o)

    def __call__(self):
        return self._outputs[0] if len(self._outputs) == 1 else self._outputs


# ----------------------------------------------------------------------------- sequence ops (LoD)
# paddle.static.nn's sequence ops ARE fluid.layers.sequence_lod's (reference
# python/paddle/static/nn/__init__.py:46-60): LoD inputs, one recorded op each.
def _seq(name):
    def f(*args, **kwargs):
        from ..fluid.layers import sequence_lod
        return getattr(sequence_lod, name)(*args, **kwargs)
    f.__name__ = name
    f.__qualname__ = name
    f.__doc__ = f"fluid.layers.sequence_lod.{name} (LoD sequence op)"
    return f


for _n in ("sequence_pool", "sequence_first_step", "sequence_last_step", "sequence_softmax", "sequence_reverse",
           "sequence_pad", "sequence_unpad", "sequence_concat", "sequence_enumerate", "sequence_expand",
           "sequence_expand_as", "sequence_reshape", "sequence_scatter", "sequence_slice", "sequence_conv"):
    globals()[_n] = _seq(_n)
