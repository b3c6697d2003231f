"""``fluid.layers`` generated activation / unary ops (reference:
python/paddle/fluid/layers/ops.py: __activations_noattr__, __unary_func__,
__inplace_unary_func__ plus softshrink, hard_shrink, cumsum, thresholded_relu, gelu, erf)."""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from ._common import T, W, register

_UNARY = {
    "sigmoid": torch.sigmoid, "silu": TF.silu, "logsigmoid": TF.logsigmoid, "tanh_shrink": lambda x: x - torch.tanh(x),
    "softplus": TF.softplus, "softsign": TF.softsign, "tanh": torch.tanh, "exp": torch.exp, "expm1": torch.expm1,
    "atan": torch.atan, "sqrt": torch.sqrt, "rsqrt": torch.rsqrt, "abs": torch.abs, "ceil": torch.ceil,
    "floor": torch.floor, "cos": torch.cos, "tan": torch.tan, "acos": torch.acos, "sin": torch.sin, "sinh": torch.sinh,
    "asin": torch.asin, "cosh": torch.cosh, "round": torch.round, "reciprocal": torch.reciprocal,
    "square": torch.square, "lgamma": torch.lgamma, "acosh": torch.acosh, "asinh": torch.asinh, "atanh": torch.atanh,
}
_INPLACE = ["exp_", "sqrt_", "rsqrt_", "ceil_", "floor_", "round_", "reciprocal_"]

__all__ = list(_UNARY) + _INPLACE + ["softshrink", "hard_shrink", "cumsum", "thresholded_relu", "gelu", "erf"]


def _make(fn, name):
    def op(x, name=None):
        return W(fn(T(x)), x)
    op.__name__ = name
    return op


def _make_inplace(fn, name):
    def op(x, name=None):
        x._t = fn(x._t)
        return x
    op.__name__ = name
    return op


for _n, _f in _UNARY.items():
    globals()[_n] = _make(_f, _n)
for _n in _INPLACE:
    globals()[_n] = _make_inplace(_UNARY[_n[:-1]], _n)


def softshrink(x, alpha=None):
    a = 0.5 if alpha is None else alpha
    t = T(x)
    return W(torch.where(t > a, t - a, torch.where(t < -a, t + a, torch.zeros_like(t))))


def hard_shrink(x, threshold=None):
    th = 0.5 if threshold is None else threshold
    t = T(x)
    return W(torch.where(t.abs() > th, t, torch.zeros_like(t)))


def cumsum(x, axis=None, exclusive=None, reverse=None):
    t = T(x)
    a = -1 if axis is None else axis
    if reverse:
        t = t.flip(a)
    out = torch.cumsum(t, a)
    if exclusive:
        out = out - t
    if reverse:
        out = out.flip(a)
    return W(out)


def thresholded_relu(x, threshold=None):
    th = 1.0 if threshold is None else threshold
    t = T(x)
    return W(torch.where(t > th, t, torch.zeros_like(t)))


def gelu(x, approximate=False):
    return W(TF.gelu(T(x), approximate="tanh" if approximate else "none"))


def erf(x, name=None):
    return W(torch.erf(T(x)))


register(globals(), [n for n in __all__ if n not in _INPLACE])
