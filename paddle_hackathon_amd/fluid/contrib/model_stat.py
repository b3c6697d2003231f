"""``fluid.contrib.model_stat.summary`` (reference python/paddle/fluid/contrib/model_stat.py:39):
PARAMs and FLOPs per op of a Program — conv2d / depthwise_conv2d, pool2d, fc / mul, batch_norm and
the activations — printed as a table with the totals (the reference counts, e.g. a conv's FLOPs
= 2 * H_out * W_out * C_out * (K_h * K_w * C_in / groups + bias)). Op types are the reference
types of the recorded ops (static/serialize.py op_reference); shapes drop the batch dim."""
from __future__ import annotations

from collections import OrderedDict

__all__ = ["summary"]

_ACTS = ("sigmoid", "tanh", "relu", "leaky_relu", "prelu")


def _prod(xs):
    n = 1
    for x in xs:
        n *= int(x)
    return n


def _summary_op(op):
    from ...static.serialize import op_reference
    from ...framework.core import Tensor
    ref = op_reference(op)
    if ref is None:
        return None
    typ, slots = ref

    def arg(slot):
        k = slots.get(slot)
        v = op.kwargs.get(k) if k is not None else None
        return v if isinstance(v, Tensor) else None

    out = next((v for v in (op.outputs if isinstance(op.outputs, (list, tuple)) else [op.outputs])
                if isinstance(v, Tensor)), None)
    if out is None:
        return None
    oshape = list(out.shape)
    if typ in ("conv2d", "depthwise_conv2d"):
        w, x = arg("Filter"), arg("Input")
        if w is None or x is None or len(oshape) != 4:
            return None
        cout, cin_g, kh, kw = list(w.shape)
        nhwc = op.kwargs.get("data_format", "NCHW") == "NHWC"
        h, wo = (oshape[1], oshape[2]) if nhwc else (oshape[2], oshape[3])
        kernel = kh * kw * cin_g
        bias = 1 if arg("Bias") is not None else 0
        return list(x.shape), oshape, cout * (kernel + bias), 2 * h * wo * cout * (kernel + bias)
    if typ == "pool2d":
        x = arg("X")
        k = op.kwargs.get("kernel_size") or op.kwargs.get("pool_size") or 1
        k = list(k) if isinstance(k, (list, tuple)) else [k, k]
        if x is None or len(oshape) != 4:
            return None
        return list(x.shape), oshape, 0, _prod(oshape[1:]) * k[0] * k[1]
    if typ in ("fc", "mul", "matmul_v2", "matmul"):
        w, x = arg("W") if typ == "fc" else arg("Y"), arg("Input") if typ == "fc" else arg("X")
        if w is None or x is None or not getattr(w, "persistable", False) or len(w.shape) != 2:
            return None
        kin, kout = list(w.shape)
        return list(x.shape), oshape, kin * kout + 1, kin * kout
    if typ in _ACTS:
        x = arg("X")
        if x is None:
            return None
        return list(x.shape), oshape, 1 if typ == "prelu" else 0, _prod(d for d in x.shape[1:])
    if typ == "batch_norm":
        x = arg("X")
        if x is None or len(x.shape) != 4:
            return None
        c = x.shape[1] if op.kwargs.get("data_format", "NCHW") != "NHWC" else x.shape[3]
        return list(x.shape), oshape, c * 2, _prod(x.shape[1:]) * 2
    return None


def summary(main_prog):
    """print the table; returns (rows, total PARAMs, total FLOPs)"""
    rows = []
    for b in main_prog.blocks:
        for op in b.ops:
            r = _summary_op(op)
            if r is None:
                continue
            from ...static.serialize import op_reference
            info = OrderedDict(type=op_reference(op)[0], input_shape=tuple(r[0][1:]), out_shape=tuple(r[1][1:]),
                               PARAMs=int(r[2]), FLOPs=int(r[3]))
            rows.append(info)
    head = ["No.", "TYPE", "INPUT", "OUTPUT", "PARAMs", "FLOPs"]
    table = [[i, o["type"], str(o["input_shape"]), str(o["out_shape"]), o["PARAMs"], o["FLOPs"]]
             for i, o in enumerate(rows)]
    widths = [max(len(str(h)), *(len(str(r[j])) for r in table)) if table else len(h) for j, h in enumerate(head)]
    sep = "+" + "+".join("-" * (w + 2) for w in widths) + "+"
    lines = [sep, "|" + "|".join(f" {h:>{w}} " for h, w in zip(head, widths)) + "|", sep]
    lines += ["|" + "|".join(f" {str(c):>{w}} " for c, w in zip(r, widths)) + "|" for r in table]
    lines.append(sep)
    tp, tf = sum(o["PARAMs"] for o in rows), sum(o["FLOPs"] for o in rows)
    print("\n".join(lines))
    print("Total PARAMs: {}({:.4f}M)".format(tp, tp / 10 ** 6))
    print("Total FLOPs: {}({:.2f}G)".format(tf, tf / 10 ** 9))
    print("Notice: \n now supported ops include [Conv, DepthwiseConv, FC(mul), BatchNorm, Pool, "
          "Activation(sigmoid, tanh, relu, leaky_relu, prelu)]")
    return rows, tp, tf
