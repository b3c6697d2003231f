"""``fluid.contrib.op_freq_statistic`` (reference python/paddle/fluid/contrib/op_frequence.py:23):
how often each op type occurs in a Program and how often each producer -> consumer pair of op
types occurs (ops writing only parameters, and parameter inputs, are not counted). Op types are
the reference types a saved program would carry (static/serialize.py op_reference), else the
recorded API name."""
from __future__ import annotations

from collections import OrderedDict

__all__ = ["op_freq_statistic"]


def _type(op):
    from ...static.serialize import op_reference, _qual_short
    r = op_reference(op)
    return r[0] if r is not None else _qual_short(op.type).rsplit(".", 1)[-1]


def op_freq_statistic(program):
    """-> (uni_op_freq, adj_2_op_freq): lists of (op type | "producer->consumer", count), most
    frequent first"""
    from ...static.program import Program
    if not isinstance(program, Program):
        raise TypeError("The input type should be Porgram. But you passed in %s" % (type(program)))
    params = {p.name for p in program.all_parameters()}
    ops = program.global_block().ops
    uni = OrderedDict()
    for op in ops:
        outs = [n for n in op.output_arg_names() if n not in params]
        if outs or not op.output_arg_names():
            t = _type(op)
            uni[t] = uni.get(t, 0) + 1
    gen = {}
    pairs = OrderedDict()
    for op in ops:
        t = _type(op)
        for n in op.input_arg_names():
            if n in params or n not in gen:
                continue
            key = gen[n][-1] + "->" + t
            pairs[key] = pairs.get(key, 0) + 1
        for n in op.output_arg_names():
            gen.setdefault(n, []).append(t)
    return (sorted(uni.items(), key=lambda kv: kv[1], reverse=True),
            sorted(pairs.items(), key=lambda kv: kv[1], reverse=True))
