"""Emit side of the ProgramDesc converters: recorded API calls whose reference op needs attributes
computed from the call (not a 1:1 renaming, see serialize._REF) — indexing, comparisons, shape
ops, search ops and the fake-quantization ops. Each emitter returns

    (reference op type, {kwarg: input slot}, output slot(s), {attr: value}, {slot: extra tensor})

or None when the call has no single-op reference form (the op is then written under its own
qualified type). Output slots: one name, a tuple of names (one output each), or one name for a
list output. Attribute names and defaults follow paddle/fluid/operators/*_op.cc:
slice_op.cc / strided_slice_op.cc (axes, starts, ends, strides, decrease_axis, infer_flags),
compare_op.cc (axis, force_cpu), expand_v2_op.cc (shape), split_op.cc (num, sections, axis),
stack_op.cc (axis), tile_op.cc (repeat_times), clip_op.cc (min, max), cum_op.cc (axis, flatten,
exclusive, reverse), arg_min_max_op_base.h (axis, keepdims, flatten, dtype), top_k_v2_op.cc
(k, axis, largest, sorted), scale_op.cc, fake_quantize_op.cc / fake_dequantize_op.cc /
quantize_linear_op.cc (bit_length, round_type, quant_axis, moving_rate, is_test, max_range)."""
from __future__ import annotations

import torch

from ..framework.core import Tensor, _wrap
from . import proto as pb

_INT_MAX = 2 ** 31 - 1


def _is_t(v):
    return isinstance(v, Tensor)


def _const(v, like=None):
    dt = like._t.dtype if isinstance(like, Tensor) and like._t.is_floating_point() else None
    return _wrap(torch.tensor(v, dtype=dt if dt is not None and isinstance(v, float) else None))


def _ints(v):
    return isinstance(v, (list, tuple)) and all(isinstance(x, int) and not isinstance(x, bool) for x in v)


def _cmp(typ):
    def emit(kw):
        x, y = kw.get("x"), kw.get("y")
        if not _is_t(x):
            return None
        extra = {} if _is_t(y) else {"Y": _const(y, x)}
        return typ, {"x": "X", "y": "Y"}, "Out", {"axis": -1, "force_cpu": False}, extra
    return emit


def _elt(typ):
    """elementwise binary op; a Python-scalar operand becomes a constant input tensor"""
    def emit(kw):
        x, y = kw.get("x"), kw.get("y")
        if not (_is_t(x) or _is_t(y)):
            return None
        extra = {}
        if not _is_t(y):
            extra["Y"] = _const(y, x)
        if not _is_t(x):
            extra["X"] = _const(x, y)
        return typ, {"x": "X", "y": "Y"}, "Out", {"axis": -1}, extra
    return emit


def _getitem(kw):
    x, idx = kw.get("x"), kw.get("idx")
    if not _is_t(x):
        return None
    rank = x._t.dim()
    items = list(idx) if isinstance(idx, tuple) else [idx]
    if sum(1 for i in items if i is Ellipsis) > 1:
        return None
    if any(i is Ellipsis for i in items):
        k = items.index(Ellipsis)
        items = items[:k] + [slice(None)] * (rank - len(items) + 1) + items[k + 1:]
    if len(items) > rank or not all(isinstance(i, (int, slice)) and not isinstance(i, bool) for i in items):
        return None
    axes, starts, ends, strides, dec = [], [], [], [], []
    for ax, it in enumerate(items):
        if isinstance(it, int):
            axes.append(ax)
            starts.append(it)
            ends.append(it + 1 if it != -1 else _INT_MAX)
            strides.append(1)
            dec.append(ax)
            continue
        if not all(v is None or (isinstance(v, int) and not isinstance(v, bool)) for v in (it.start, it.stop, it.step)):
            return None
        if it.start is None and it.stop is None and it.step in (None, 1):
            continue
        step = 1 if it.step is None else it.step
        axes.append(ax)
        strides.append(step)
        if step > 0:
            starts.append(0 if it.start is None else it.start)
            ends.append(_INT_MAX if it.stop is None else it.stop)
        else:
            starts.append(-1 if it.start is None else it.start)
            ends.append(-_INT_MAX if it.stop is None else it.stop)
    if not axes:   # x[:] / x[...]: a copy
        return "assign", {"x": "X"}, "Out", {}, {}
    if all(s == 1 for s in strides):
        return "slice", {"x": "Input"}, "Out", {"axes": axes, "starts": starts, "ends": ends, "decrease_axis": dec,
                                                "infer_flags": [1] * len(axes)}, {}
    return "strided_slice", {"x": "Input"}, "Out", {"axes": axes, "starts": starts, "ends": ends, "strides": strides,
                                                    "decrease_axis": dec, "infer_flags": [1] * len(axes)}, {}


def _expand(kw):
    s = kw.get("shape")
    if not _ints(s):
        return None
    return "expand_v2", {"x": "X"}, "Out", {"shape": list(s)}, {}


def _split(kw):
    n, ax = kw.get("num_or_sections"), kw.get("axis", 0)
    if not isinstance(ax, int):
        return None
    if isinstance(n, int):
        return "split", {"x": "X"}, "Out", {"num": n, "axis": ax}, {}
    if _ints(n):
        return "split", {"x": "X"}, "Out", {"num": 0, "sections": list(n), "axis": ax}, {}
    return None


def _stack(kw):
    return "stack", {"x": "X"}, "Y", {"axis": int(kw.get("axis", 0))}, {}


def _tile(kw):
    r = kw.get("repeat_times")
    if not _ints(r):
        return None
    return "tile", {"x": "X"}, "Out", {"repeat_times": list(r)}, {}


def _where(kw):
    c, x, y = kw.get("condition"), kw.get("x"), kw.get("y")
    if x is None and y is None:
        return "where_index", {"condition": "Condition"}, "Out", {}, {}
    extra = {}
    if not _is_t(x):
        extra["X"] = _const(x, y)
    if not _is_t(y):
        extra["Y"] = _const(y, x)
    return "where", {"condition": "Condition", "x": "X", "y": "Y"}, "Out", {}, extra


def _clip(kw):
    lo, hi = kw.get("min"), kw.get("max")
    at, extra = {}, {}
    for name, v, d in (("min", lo, -3.4028234663852886e38), ("max", hi, 3.4028234663852886e38)):
        if v is None:
            at[name] = d
        elif _is_t(v):
            at[name] = d   # the tensor goes to the Min / Max slot
        else:
            at[name] = float(v)
    return "clip", {"x": "X", "min": "Min", "max": "Max"}, "Out", at, extra


def _cumsum(kw):
    ax = kw.get("axis")
    return "cumsum", {"x": "X"}, "Out", {"axis": -1 if ax is None else int(ax), "flatten": ax is None,
                                         "exclusive": False, "reverse": False}, {}


def _arg(typ):
    def emit(kw):
        ax = kw.get("axis")
        from ..framework.core import convert_dtype
        dt = pb.vartype_of(convert_dtype(kw.get("dtype", "int64")))
        return typ, {"x": "X"}, "Out", {"axis": 0 if ax is None else int(ax), "keepdims": bool(kw.get("keepdim")),
                                        "flatten": ax is None, "dtype": dt}, {}
    return emit


def _topk(kw):
    k = kw.get("k")
    if not isinstance(k, int):
        return None
    ax = kw.get("axis")
    return "top_k_v2", {"x": "X"}, ("Out", "Indices"), {"k": k, "axis": -1 if ax is None else int(ax),
                                                         "largest": bool(kw.get("largest", True)),
                                                         "sorted": bool(kw.get("sorted", True))}, {}


def _neg(kw):
    return "scale", {"x": "X"}, "Out", {"scale": -1.0, "bias": 0.0, "bias_after_scale": True}, {}


def _cast(kw):
    x, dt = kw.get("x"), kw.get("dtype")
    if not _is_t(x):
        return None
    from ..framework.core import convert_dtype
    return "cast", {"x": "X"}, "Out", {"in_dtype": pb.vartype_of(x._t.dtype),
                                       "out_dtype": pb.vartype_of(convert_dtype(dt))}, {}


# ------------------------------------------------------------------------------- quantization
def _qdq_abs_max(kw):
    return "fake_quantize_dequantize_abs_max", {"x": "X"}, ("Out", "OutScale"), \
        {"bit_length": int(kw.get("bit_length", 8)), "round_type": int(kw.get("round_type", 1))}, {}


def _q_abs_max(kw):
    return "fake_quantize_abs_max", {"x": "X"}, ("Out", "OutScale"), \
        {"bit_length": int(kw.get("bit_length", 8)), "round_type": int(kw.get("round_type", 1))}, {}


def _qdq_channel(typ):
    def emit(kw):
        return typ, {"x": "X"}, ("Out", "OutScale"), {"bit_length": int(kw.get("bit_length", 8)),
                                                       "quant_axis": int(kw.get("quant_axis", 0)),
                                                       "round_type": int(kw.get("round_type", 1))}, {}
    return emit


def _qdq_moving(typ):
    def emit(kw):
        return typ, {"x": "X", "in_scale": "InScale", "in_state": "InState", "in_accum": "InAccum"}, "Out", \
            {"bit_length": int(kw.get("bit_length", 8)), "moving_rate": float(kw.get("moving_rate", 0.9)),
             "is_test": bool(kw.get("is_test", False)), "round_type": int(kw.get("round_type", 1))}, \
            {"@out:OutScale": kw.get("in_scale"), "@out:OutState": kw.get("in_state"),
             "@out:OutAccum": kw.get("in_accum")}
    return emit


def _ma_scale(kw):
    return "moving_average_abs_max_scale", {"x": "X", "in_scale": "InScale", "in_state": "InState",
                                            "in_accum": "InAccum"}, "Out", \
        {"moving_rate": float(kw.get("moving_rate", 0.9)), "is_test": bool(kw.get("is_test", False))}, \
        {"@out:OutScale": kw.get("in_scale"), "@out:OutState": kw.get("in_state"),
         "@out:OutAccum": kw.get("in_accum")}


def _qdq_fixed(kw):
    """a frozen (calibrated) quant-dequant: the reference writes it as the moving-average op with
    is_test = True reading the stored scale (per tensor), or the channel-wise op (per channel)"""
    s = kw.get("scale")
    if _is_t(s) and s._t.numel() > 1:
        return "fake_channel_wise_quantize_dequantize_abs_max", {"x": "X", "scale": "InScale"}, "Out", \
            {"bit_length": int(kw.get("bit_length", 8)), "quant_axis": int(kw.get("quant_axis") or 0),
             "round_type": int(kw.get("round_type", 1))}, {}
    return "fake_quantize_dequantize_moving_average_abs_max", {"x": "X", "scale": "InScale"}, "Out", \
        {"bit_length": int(kw.get("bit_length", 8)), "moving_rate": 0.9, "is_test": True,
         "round_type": int(kw.get("round_type", 1))}, {}


def _q_linear(typ):
    def emit(kw):
        at = {"bit_length": int(kw.get("bit_length", 8)), "quant_axis": int(kw.get("quant_axis", -1))}
        if typ == "quantize_linear":
            at["round_type"] = int(kw.get("round_type", 0))
        return typ, {"x": "X", "scale": "Scale", "zero_point": "ZeroPoint"}, "Y", at, {}
    return emit


def _deq_max_abs(kw):
    return "fake_dequantize_max_abs", {"x": "X", "scale": "Scale"}, "Out", \
        {"max_range": float(kw.get("max_range", 127.0))}, {}


def _ch_deq(kw):
    return "fake_channel_wise_dequantize_max_abs", {"x": "X", "scales": "Scales"}, "Out", \
        {"quant_bits": [int(b) for b in kw.get("quant_bits", (8,))], "quant_axis": int(kw.get("quant_axis", 0))}, {}


# ------------------------------------------------------------------------------- LoD sequence ops
# (sequence_ops/sequence_*_op.cc: slot and attribute names)
def _seq_pool(pooltype=None):
    def emit(kw):
        pt = (pooltype or kw.get("pool_type", "average")).upper()
        return "sequence_pool", {"input": "X"}, "Out", {"pooltype": pt, "is_test": bool(kw.get("is_test", False)),
                                                        "pad_value": float(kw.get("pad_value", 0.0))}, {}
    return emit


def _seq_conv(kw):
    if kw.get("bias") is not None:
        return None
    return "sequence_conv", {"input": "X", "filter": "Filter"}, "Out", \
        {"contextLength": int(kw.get("context_length", 3)), "contextStart": int(kw.get("context_start", -1)),
         "contextStride": int(kw.get("context_stride", 1)), "paddingTrainable": False}, {}


def _seq_pad(kw):
    pv = kw.get("pad_value")
    ml = kw.get("maxlen")
    return "sequence_pad", {"x": "X", "pad_value": "PadValue"}, ("Out", "Length"), \
        {"padded_length": -1 if ml is None else int(ml)}, ({} if _is_t(pv) else {"PadValue": _const(pv)})


def _seq_mask(kw):
    from ..framework.core import convert_dtype
    ml = kw.get("maxlen")
    if _is_t(ml):
        return None
    return "sequence_mask", {"x": "X"}, "Y", {"maxlen": -1 if ml is None else int(ml),
                                              "out_dtype": pb.vartype_of(convert_dtype(kw.get("dtype", "int64")))}, {}


def _lookup_v1(kw):
    pad = kw.get("padding_idx")
    return "lookup_table", {"input": "Ids", "w": "W"}, "Out", \
        {"padding_idx": -1 if pad is None else int(pad), "is_sparse": False, "is_distributed": False}, {}


_S = "fluid.layers.sequence_lod."
_SEQ = {
    _S + "sequence_pool": _seq_pool(),
    _S + "sequence_first_step": _seq_pool("FIRST"),
    _S + "sequence_last_step": _seq_pool("LAST"),
    _S + "sequence_conv_op": _seq_conv,
    _S + "sequence_softmax": lambda kw: ("sequence_softmax", {"input": "X"}, "Out", {}, {}),
    _S + "sequence_expand": lambda kw: ("sequence_expand", {"x": "X", "y": "Y"}, "Out",
                                        {"ref_level": int(kw.get("ref_level", -1))}, {}),
    _S + "sequence_expand_as": lambda kw: ("sequence_expand_as", {"x": "X", "y": "Y"}, "Out", {}, {}),
    _S + "sequence_pad": _seq_pad,
    _S + "sequence_unpad": lambda kw: ("sequence_unpad", {"x": "X", "length": "Length"}, "Out", {}, {}),
    _S + "sequence_reverse": lambda kw: ("sequence_reverse", {"x": "X"}, "Y", {}, {}),
    _S + "sequence_concat": lambda kw: ("sequence_concat", {"input": "X"}, "Out", {}, {}),
    _S + "sequence_reshape": lambda kw: ("sequence_reshape", {"input": "X"}, "Out",
                                         {"new_dim": int(kw.get("new_dim"))}, {}),
    _S + "sequence_mask": _seq_mask,
    _S + "sequence_enumerate": lambda kw: ("sequence_enumerate", {"input": "X"}, "Out",
                                           {"win_size": int(kw.get("win_size")),
                                            "pad_value": int(kw.get("pad_value", 0))}, {}),
    _S + "sequence_slice": lambda kw: ("sequence_slice", {"input": "X", "offset": "Offset", "length": "Length"},
                                       "Out", {}, {}),
    _S + "sequence_scatter": lambda kw: ("sequence_scatter", {"input": "X", "index": "Ids", "updates": "Updates"},
                                         "Out", {}, {}),
    "fluid.layers.nn._lookup_v1": _lookup_v1,
}

# ------------------------------------------------------------------------------- activations
# (activation_op.cc: the 2.x function's arguments renamed to the 1.x op's attributes)
def _act(typ, **attrs):
    """``attrs``: reference attr -> (our kwarg, default) or a constant"""
    def emit(kw):
        if kw.get("dtype") is not None:
            return None
        at = {a: (float(kw.get(v[0], v[1])) if isinstance(v, tuple) else v) for a, v in attrs.items()}
        return typ, {"x": "X"}, "Out", at, {}
    return emit


_A = "nn.functional.activation."
_ACT = {
    _A + "tanh": _act("tanh"),
    _A + "leaky_relu": _act("leaky_relu", alpha=("negative_slope", 0.01)),
    _A + "elu": _act("elu", alpha=("alpha", 1.0)),
    _A + "relu6": _act("relu6", threshold=6.0),
    _A + "hardswish": _act("hard_swish", threshold=6.0, scale=6.0, offset=3.0),
    _A + "hardsigmoid": _act("hard_sigmoid", slope=("slope", 0.1666667), offset=("offset", 0.5)),
    _A + "softplus": _act("softplus", beta=("beta", 1.0), threshold=("threshold", 20.0)),
    _A + "softshrink": _act("softshrink", **{"lambda": ("threshold", 0.5)}),
    _A + "hardshrink": _act("hard_shrink", threshold=("threshold", 0.5)),
    _A + "thresholded_relu": _act("thresholded_relu", threshold=("threshold", 1.0)),
    _A + "swish": _act("swish", beta=1.0),
    _A + "mish": _act("mish"),
    _A + "selu": _act("selu", scale=("scale", 1.0507009873554805), alpha=("alpha", 1.6732632423543772)),
    _A + "tanhshrink": _act("tanh_shrink"),
    _A + "log_sigmoid": _act("logsigmoid"),
    _A + "softsign": _act("softsign"),
    _A + "hardtanh": _act("brelu", t_min=("min", -1.0), t_max=("max", 1.0)),
    _A + "log_softmax": lambda kw: None if kw.get("dtype") is not None else
    ("log_softmax", {"x": "X"}, "Out", {"axis": int(kw.get("axis", -1))}, {}),
    **{"tensor.math." + n: _act(n) for n in ("log", "abs", "sin", "cos", "tan", "floor", "ceil", "rsqrt", "square",
                                             "reciprocal", "sign", "erf", "round", "log2", "log10", "log1p", "expm1",
                                             "atan", "asin", "acos", "sinh", "cosh")},
}

_RU_SLOTS = {"x": "X", "filter_x": "FilterX", "scale_x": "ScaleX", "bias_x": "BiasX", "mean_x": "MeanX",
             "var_x": "VarX", "z": "Z", "filter_z": "FilterZ", "scale_z": "ScaleZ", "bias_z": "BiasZ",
             "mean_z": "MeanZ", "var_z": "VarZ"}


def _resnet_unit(kw):
    """resnet_unit_op.cc: the reference filter layout only (OHWI for NHWC, OIHW for NCHW)"""
    fmt = kw.get("data_format", "NHWC")
    if kw.get("filter_layout") not in (None, "OHWI" if fmt == "NHWC" else "OIHW"):
        return None
    return "resnet_unit", dict(_RU_SLOTS), "Y", {
        "stride": int(kw["stride"]), "stride_z": int(kw["stride_z"]), "padding": int(kw["padding"]),
        "dilation": int(kw["dilation"]), "group": int(kw["groups"]), "momentum": float(kw["momentum"]),
        "epsilon": float(kw["eps"]), "data_format": fmt, "fuse_add": bool(kw["fuse_add"]),
        "has_shortcut": bool(kw["has_shortcut"]), "use_global_stats": bool(kw["use_global_stats"]),
        "is_test": bool(kw["is_test"]), "act_type": kw.get("act") or "identity"}, {}


def _nonzero(kw):
    """paddle.nonzero -> where_index (Condition -> Out [-1, rank] int64)"""
    if kw.get("as_tuple") or not _is_t(kw.get("x")):
        return None
    return "where_index", {"x": "Condition"}, "Out", {}, {}


def _fluid_where(kw):
    return "where_index", {"condition": "Condition"}, "Out", {}, {}


def _masked_select(kw):
    return "masked_select", {"x": "X", "mask": "Mask"}, "Y", {}, {}


def _unique(kw):
    """unique_op.cc: Out, then Indices / Index (inverse) / Counts as requested (is_sorted = True,
    the 2.x paddle.unique form)"""
    outs = ["Out"] + [s for f, s in (("return_index", "Indices"), ("return_inverse", "Index"),
                                       ("return_counts", "Counts")) if kw.get(f)]
    axis = kw.get("axis")
    return "unique", {"x": "X"}, tuple(outs) if len(outs) > 1 else "Out", {
        "dtype": pb.vartype_of(_dtype(kw.get("dtype", "int64"))), "return_index": bool(kw.get("return_index")),
        "return_inverse": bool(kw.get("return_inverse")), "return_counts": bool(kw.get("return_counts")),
        "axis": [] if axis is None else [int(axis)], "is_sorted": True}, {}


def _dtype(d):
    from ..framework.core import convert_dtype
    return convert_dtype(d) or torch.int64


def _edit_distance(kw):
    if kw.get("ignored_tokens"):
        return None   # the reference layer erases them with a sequence_erase op first
    return "edit_distance", {"input": "Hyps", "label": "Refs", "input_length": "HypsLength",
                             "label_length": "RefsLength"}, ("Out", "SequenceNum"), {
        "normalized": bool(kw.get("normalized", True))}, {}


def _pair(v, n=2):
    if isinstance(v, int) and not isinstance(v, bool):
        return [v] * n
    if _ints(v) and len(v) == n:
        return list(v)
    raise ValueError(v)


def _paddings(p):
    """(paddings, padding_algorithm) of conv_op.cc / pool_op.cc from a 2.x ``padding`` argument"""
    if isinstance(p, str):
        return [0, 0], p.upper()
    if isinstance(p, int) and not isinstance(p, bool):
        return [p, p], "EXPLICIT"
    if _ints(p) and len(p) in (2, 4):
        return list(p), "EXPLICIT"
    if isinstance(p, (list, tuple)) and len(p) == 4 and all(_ints(q) and len(q) == 2 for q in p):
        return [x for q in p[2:] for x in q], "EXPLICIT"   # NCHW pairs: the spatial two
    raise ValueError(p)


def _conv2d(kw):
    """conv_op.cc: strides / paddings / dilations as INTS (2.x F.conv2d's static branch)"""
    if not (_is_t(kw.get("x")) and _is_t(kw.get("weight"))):
        return None
    pads, algo = _paddings(kw.get("padding", 0))
    slots = {"x": "Input", "weight": "Filter"}
    if _is_t(kw.get("bias")):
        slots["bias"] = "Bias"
    groups = int(kw.get("groups", 1))
    w = kw["weight"]
    depthwise = groups > 1 and groups == int(w._t.shape[0]) and int(w._t.shape[1]) == 1
    return "depthwise_conv2d" if depthwise else "conv2d", slots, "Output", {
        "strides": _pair(kw.get("stride", 1)), "paddings": pads, "padding_algorithm": algo,
        "dilations": _pair(kw.get("dilation", 1)), "groups": groups,
        "data_format": kw.get("data_format", "NCHW"), "use_cudnn": True}, {}


def _pool2d(kind):
    def emit(kw):
        if not _is_t(kw.get("x")) or kw.get("return_mask") or kw.get("divisor_override"):
            return None
        k = _pair(kw["kernel_size"])
        st = kw.get("stride")
        pads, algo = _paddings(kw.get("padding", 0))
        return "pool2d", {"x": "X"}, "Out", {
            "pooling_type": kind, "ksize": k, "strides": k if st is None else _pair(st), "paddings": pads,
            "padding_algorithm": algo, "global_pooling": False, "adaptive": False,
            "ceil_mode": bool(kw.get("ceil_mode", False)), "exclusive": bool(kw.get("exclusive", True)),
            "data_format": kw.get("data_format", "NCHW"), "use_cudnn": True}, {}
    return emit


def _adaptive_pool2d(kind):
    def emit(kw):
        if not _is_t(kw.get("x")) or kw.get("return_mask"):
            return None
        os_ = kw["output_size"]
        if isinstance(os_, (list, tuple)) and any(o is None for o in os_):
            return None
        return "pool2d", {"x": "X"}, "Out", {
            "pooling_type": kind, "ksize": _pair(os_), "strides": [1, 1], "paddings": [0, 0],
            "padding_algorithm": "EXPLICIT", "global_pooling": False, "adaptive": True, "ceil_mode": False,
            "exclusive": True, "data_format": kw.get("data_format", "NCHW"), "use_cudnn": True}, {}
    return emit


_Q = "nn.quant.ops."
EMIT = {
    "nn.functional.conv.conv2d": _conv2d,
    "nn.functional.pooling.max_pool2d": _pool2d("max"),
    "nn.functional.pooling.avg_pool2d": _pool2d("avg"),
    "nn.functional.pooling.adaptive_avg_pool2d": _adaptive_pool2d("avg"),
    "nn.functional.pooling.adaptive_max_pool2d": _adaptive_pool2d("max"),
    "fluid.layers.loss.edit_distance": _edit_distance,
    "tensor.manipulation.nonzero": _nonzero,
    "tensor.manipulation.masked_select": _masked_select,
    "tensor.manipulation.unique": _unique,
    "fluid.layers.nn.where": _fluid_where,
    "incubate.operators.resnet_unit.resnet_unit": _resnet_unit,
    **_SEQ,
    **_ACT,
    **{f"tensor.logic.{n}": _cmp(n) for n in ("greater_than", "greater_equal", "less_than", "less_equal", "equal",
                                               "not_equal")},
    **{f"tensor.math.{n}": _elt(t) for n, t in (("add", "elementwise_add"), ("subtract", "elementwise_sub"),
                                                ("multiply", "elementwise_mul"), ("divide", "elementwise_div"),
                                                ("maximum", "elementwise_max"), ("minimum", "elementwise_min"),
                                                ("pow", "elementwise_pow"))},
    "tensor.getitem": _getitem,
    "tensor.manipulation.expand": _expand,
    "tensor.manipulation.broadcast_to": _expand,
    "tensor.manipulation.split": _split,
    "tensor.manipulation.stack": _stack,
    "tensor.manipulation.tile": _tile,
    "tensor.manipulation.where": _where,
    "tensor.math.clip": _clip,
    "tensor.math.cumsum": _cumsum,
    "tensor.search.argmax": _arg("arg_max"),
    "tensor.search.argmin": _arg("arg_min"),
    "tensor.search.topk": _topk,
    "tensor.math.neg": _neg,
    "tensor.manipulation.cast": _cast,
    _Q + "fake_quantize_dequantize_abs_max": _qdq_abs_max,
    _Q + "fake_quantize_abs_max": _q_abs_max,
    _Q + "fake_channel_wise_quantize_dequantize_abs_max": _qdq_channel("fake_channel_wise_quantize_dequantize_abs_max"),
    _Q + "fake_channel_wise_quantize_abs_max": _qdq_channel("fake_channel_wise_quantize_abs_max"),
    _Q + "fake_quantize_dequantize_moving_average_abs_max":
        _qdq_moving("fake_quantize_dequantize_moving_average_abs_max"),
    _Q + "fake_quantize_moving_average_abs_max": _qdq_moving("fake_quantize_moving_average_abs_max"),
    _Q + "moving_average_abs_max_scale": _ma_scale,
    _Q + "fake_quantize_dequantize_fixed_scale": _qdq_fixed,
    _Q + "quantize_linear": _q_linear("quantize_linear"),
    _Q + "dequantize_linear": _q_linear("dequantize_linear"),
    _Q + "fake_dequantize_max_abs": _deq_max_abs,
    _Q + "fake_channel_wise_dequantize_max_abs": _ch_deq,
}


def spec(short, op):
    f = EMIT.get(short)
    if f is None or op.args:
        return None
    try:
        return f(op.kwargs)
    except (TypeError, ValueError):
        return None


# ------------------------------------------------------------------------------- composites
# calls whose reference static graph is SEVERAL ops (reference: the static branch of the Python
# function appends them one by one): written as those ops with intermediate variables; in a
# training program their grad op becomes the parts' grad ops in reverse order (static/ref_train.py)

def _tmp_var(name, like, shape, dtype=None):
    import torch
    from .program import Variable
    meta = torch.empty([1 if (s is None or s < 0) else int(s) for s in shape], dtype=dtype or like._t.dtype,
                       device="meta")
    return Variable(None, meta, name=name, declared_shape=[(-1 if s is None else int(s)) for s in shape])


def _ce_composite(op):
    """nn/functional/loss.py cross_entropy (static branch, hard labels, softmax, no weight or label
    smoothing, ignore_index < 0): softmax_with_cross_entropy -> (Softmax, Loss), then the mean
    (reduce_mean over all elements) or sum (reduce_sum)"""
    kw = op.kwargs
    if (op.args or kw.get("soft_label") or not kw.get("use_softmax", True) or kw.get("weight") is not None
            or kw.get("label_smoothing", 0.0) or int(kw.get("ignore_index", -100)) >= 0
            or kw.get("reduction", "mean") not in ("mean", "sum")):
        return None
    x, lab, out = kw.get("input"), kw.get("label"), op.outputs
    if not (_is_t(x) and _is_t(lab)) or isinstance(out, (list, tuple)):
        return None
    axis = int(kw.get("axis", -1))
    shape = list(getattr(x, "declared_shape", None) or x.shape)
    lshape = list(shape)
    lshape[axis] = 1
    sm = _tmp_var(out.name + "@swce_softmax", x, shape)
    loss = _tmp_var(out.name + "@swce_loss", x, lshape)
    red = "reduce_mean" if kw.get("reduction", "mean") == "mean" else "reduce_sum"
    return [("softmax_with_cross_entropy", {"Logits": [x], "Label": [lab]}, {"Softmax": [sm], "Loss": [loss]},
             {"soft_label": False, "ignore_index": int(kw.get("ignore_index", -100)), "numeric_stable_mode": True,
              "axis": axis, "use_softmax": True}),
            (red, {"X": [loss]}, {"Out": [out]}, {"dim": [0], "keep_dim": False, "reduce_all": True})]


def _dropout_composite(op):
    """dropout_op.cc: Out and the uint8 Mask (what dropout_grad multiplies by), is_test from our
    ``training`` flag, implementation upscale_in_train / downgrade_in_infer"""
    import torch
    kw = op.kwargs
    x, out, p = kw.get("x"), op.outputs, kw.get("p", 0.5)
    if op.args or not _is_t(x) or kw.get("axis") is not None or _is_t(p) or isinstance(out, (list, tuple)):
        return None
    mode = kw.get("mode", "upscale_in_train")
    mask = _tmp_var(out.name + "@dropout_mask", x, list(getattr(x, "declared_shape", None) or x.shape), torch.uint8)
    return [("dropout", {"X": [x]}, {"Out": [out], "Mask": [mask]},
             {"dropout_prob": float(p), "is_test": not kw.get("training", True), "fix_seed": False, "seed": 0,
              "dropout_implementation": "upscale_in_train" if mode == "upscale_in_train" else "downgrade_in_infer"})]


COMPOSITE = {"nn.functional.loss.cross_entropy": _ce_composite, "nn.functional.common.dropout": _dropout_composite}
# written this way in training programs only (inference programs keep the call, which the
# inference passes rewrite, e.g. delete_dropout_op_pass)
TRAIN_ONLY = {"nn.functional.common.dropout"}


def composite(w, short, op):
    """the op's parts [(type, {slot: [tensors]}, {slot: [Variables]}, attrs)] (cached per writer, so
    the forward and its grad op see the same intermediates) or None"""
    f = COMPOSITE.get(short)
    if f is None or (short in TRAIN_ONLY and not getattr(w, "train", False)):
        return None
    cache = w.__dict__.setdefault("_composite", {})
    if id(op) not in cache:
        cache[id(op)] = (op, f(op))
    return cache[id(op)][1]


def write_parts(w, parts, block_msg, role=None):
    from .serialize import _set_attr
    for typ, ins, outs, attrs in parts:
        msg = block_msg.ops.add()
        msg.type = typ
        for k, v in attrs.items():
            _set_attr(msg, k, v)
        if role is not None and "op_role" not in attrs:
            _set_attr(msg, "op_role", role)
        for slot, ts in ins.items():
            s = msg.inputs.add()
            s.parameter = slot
            s.arguments.extend(w.tensor_name(t) for t in ts)
        for slot, ts in outs.items():
            s = msg.outputs.add()
            s.parameter = slot
            s.arguments.extend(w.tensor_name(t) for t in ts)
