"""Elementwise / reduction math ops (reference: python/paddle/tensor/math.py,
python/paddle/tensor/stat.py, phi/kernels/{elementwise,reduce,activation}*).

Elementwise and reduction ops execute as PyTorch-ROCm kernels on HIP; the
fused hot paths (norms, softmax-CE, optimizers, attention) are our own HIP
kernels in ``paddle_hackathon_amd.ops``.
"""
from __future__ import annotations

import builtins
import functools
import math as _pymath

import numpy as np
import torch

from ..framework import core as _core
from ..framework.core import Tensor
from ..framework.dispatch import register_ops
from ._helpers import _u, _w, _axis, _int_list, _scalar, _to_t, convert_dtype

__all__ = []


def _export(fn):
    __all__.append(fn.__name__)
    return fn


# ----------------------------------------------------------------------------
# unary elementwise
# ----------------------------------------------------------------------------
def _round_half_away(t):
    """reference RoundFunctor is Eigen ``x.round()`` = std::round: halves go away from zero
    (torch.round rounds them to even)"""
    if not t.is_floating_point():
        return t
    tr = torch.trunc(t)
    return torch.where((t - tr).abs() == 0.5, tr + torch.sign(t), torch.round(t))


_UNARY = {
    "abs": torch.abs, "acos": torch.acos, "asin": torch.asin, "atan": torch.atan,
    "acosh": torch.acosh, "asinh": torch.asinh, "atanh": torch.atanh,
    "ceil": torch.ceil, "cos": torch.cos, "cosh": torch.cosh, "exp": torch.exp,
    "expm1": torch.expm1, "floor": torch.floor, "log": torch.log, "log2": torch.log2,
    "log10": torch.log10, "log1p": torch.log1p, "reciprocal": torch.reciprocal,
    "round": _round_half_away, "rsqrt": torch.rsqrt, "sign": torch.sign, "sin": torch.sin,
    "sinh": torch.sinh, "sqrt": torch.sqrt, "square": torch.square, "tan": torch.tan,
    "tanh": torch.tanh, "erf": torch.erf, "erfinv": torch.erfinv, "lgamma": torch.lgamma,
    "digamma": torch.digamma, "trunc": torch.trunc, "neg": torch.neg, "conj": torch.conj,
    "sigmoid": torch.sigmoid, "frac": torch.frac, "rad2deg": torch.rad2deg,
    "deg2rad": torch.deg2rad, "angle": torch.angle, "i0": torch.i0,
}
_INPLACE_UNARY = ["ceil", "exp", "floor", "reciprocal", "round", "rsqrt", "sqrt", "tanh",
                  "erfinv", "abs", "sigmoid", "sin", "cos", "log", "neg", "square"]


def _make_unary(name, f):
    def op(x, name=None):
        return _w(f(x._t if isinstance(x, Tensor) else torch.as_tensor(x)))
    op.__name__ = name
    op.__qualname__ = name
    return op


def _make_inplace(name):
    tf = getattr(torch.Tensor, name + "_")
    if name == "round":
        def tf(t):
            return t.copy_(_round_half_away(t))

    def op(x, name=None):
        tf(x._t)
        return x
    op.__name__ = name + "_"
    op.__qualname__ = name + "_"
    return op


for _n, _f in _UNARY.items():
    globals()[_n] = _make_unary(_n, _f)
    __all__.append(_n)
for _n in _INPLACE_UNARY:
    globals()[_n + "_"] = _make_inplace(_n)
    __all__.append(_n + "_")


@_export
def real(x, name=None):
    return _w(torch.real(_u(x)))


@_export
def imag(x, name=None):
    return _w(torch.imag(_u(x)))


@_export
def logit(x, eps=None, name=None):
    return _w(torch.logit(_u(x), eps))


@_export
def stanh(x, scale_a=0.67, scale_b=1.7159, name=None):
    return _w(scale_b * torch.tanh(scale_a * _u(x)))


@_export
def isfinite(x, name=None):
    return _w(torch.isfinite(_u(x)))


@_export
def isinf(x, name=None):
    return _w(torch.isinf(_u(x)))


@_export
def isnan(x, name=None):
    return _w(torch.isnan(_u(x)))


@_export
def nan_to_num(x, nan=0.0, posinf=None, neginf=None, name=None):
    return _w(torch.nan_to_num(_u(x), nan, posinf, neginf))


# ----------------------------------------------------------------------------
# binary elementwise
# ----------------------------------------------------------------------------
def _bin(x, y):
    xt = x._t if isinstance(x, Tensor) else x
    yt = y._t if isinstance(y, Tensor) else y
    if isinstance(xt, np.ndarray):
        xt = torch.from_numpy(xt).to(yt.device)
    if isinstance(yt, np.ndarray):
        yt = torch.from_numpy(yt).to(xt.device)
    if not isinstance(xt, torch.Tensor):
        xt = torch.as_tensor(xt, dtype=yt.dtype if isinstance(xt, float) and yt.is_floating_point() else None, device=yt.device)
    return xt, yt


@_export
def add(x, y, name=None):
    xt, yt = _bin(x, y)
    return _w(torch.add(xt, yt))


@_export
def subtract(x, y, name=None):
    xt, yt = _bin(x, y)
    return _w(torch.sub(xt, yt))


@_export
def multiply(x, y, name=None):
    xt, yt = _bin(x, y)
    return _w(torch.mul(xt, yt))


@_export
def divide(x, y, name=None):
    xt, yt = _bin(x, y)
    if not xt.is_floating_point() and not xt.is_complex() and (not isinstance(yt, torch.Tensor) or not yt.is_floating_point()) and not isinstance(yt, float):
        return _w(torch.div(xt, yt, rounding_mode="trunc"))
    return _w(torch.div(xt, yt))


@_export
def floor_divide(x, y, name=None):
    """Truncating division, as the reference kernel: FloorDivideFunctor returns trunc(a / b)
    (phi/kernels/funcs/elementwise_functor.h:555-561), so floor_divide(-7, 2) == -3."""
    xt, yt = _bin(x, y)
    if not torch.is_floating_point(xt) and bool((yt == 0).any()):
        raise ZeroDivisionError("floor_divide: divisor contains zero")
    return _w(torch.div(xt, yt, rounding_mode="trunc"))


@_export
def remainder(x, y, name=None):
    xt, yt = _bin(x, y)
    return _w(torch.remainder(xt, yt))


mod = remainder
floor_mod = remainder
__all__ += ["mod", "floor_mod"]


@_export
def pow(x, y, name=None):
    xt, yt = _bin(x, y)
    return _w(torch.pow(xt, yt))


@_export
def maximum(x, y, name=None):
    xt, yt = _bin(x, y)
    return _w(torch.maximum(xt, yt))


@_export
def minimum(x, y, name=None):
    xt, yt = _bin(x, y)
    return _w(torch.minimum(xt, yt))


@_export
def fmax(x, y, name=None):
    return _w(torch.fmax(_u(x), _u(y)))


@_export
def fmin(x, y, name=None):
    return _w(torch.fmin(_u(x), _u(y)))


@_export
def atan2(x, y, name=None):
    return _w(torch.atan2(_u(x), _u(y)))


@_export
def heaviside(x, y, name=None):
    return _w(torch.heaviside(_u(x), _u(y)))


@_export
def gcd(x, y, name=None):
    return _w(torch.gcd(_u(x), _u(y)))


@_export
def lcm(x, y, name=None):
    return _w(torch.lcm(_u(x), _u(y)))


@_export
def hypot(x, y, name=None):
    return _w(torch.hypot(_u(x), _u(y)))


@_export
def lerp(x, y, weight, name=None):
    return _w(torch.lerp(_u(x), _u(y), _to_t(weight)))


@_export
def lerp_(x, y, weight, name=None):
    x._t.lerp_(_u(y), _to_t(weight))
    return x


def _inplace_bin(tname):
    def op(x, y, name=None):
        getattr(x._t, tname)(_to_t(y, x._t))
        return x
    return op


add_ = _inplace_bin("add_")
subtract_ = _inplace_bin("sub_")
multiply_ = _inplace_bin("mul_")
divide_ = _inplace_bin("div_")
for _n in ("add_", "subtract_", "multiply_", "divide_"):
    globals()[_n].__name__ = _n
    __all__.append(_n)


@_export
def scale(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    t = _u(x)
    s = _scalar(scale)
    if bias_after_scale:
        out = t * s + bias if bias else t * s
    else:
        out = (t + bias) * s
    if out.dtype != t.dtype:
        out = out.to(t.dtype)
    if act is not None:
        from ..nn import functional as F
        return getattr(F, act)(_w(out))
    return _w(out)


@_export
def scale_(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    with torch.no_grad() if x._t.is_leaf and x._t.requires_grad else _nullctx():
        if bias_after_scale:
            x._t.mul_(_scalar(scale)).add_(bias)
        else:
            x._t.add_(bias).mul_(_scalar(scale))
    return x


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


@_export
def increment(x, value=1.0, name=None):
    with torch.no_grad():
        x._t.add_(value)
    return x


@_export
def clip(x, min=None, max=None, name=None):
    mn = _scalar(min)
    mx = _scalar(max)
    return _w(torch.clamp(_u(x), mn, mx))


@_export
def clip_(x, min=None, max=None, name=None):
    x._t.clamp_(_scalar(min), _scalar(max))
    return x


@_export
def add_n(inputs, name=None):
    if isinstance(inputs, Tensor):
        return inputs
    ts = [_u(t) for t in inputs]
    out = ts[0]
    for t in ts[1:]:
        out = out + t
    return _w(out)


@_export
def multiplex(inputs, index, name=None):
    stacked = torch.stack([_u(t) for t in inputs], 0)
    idx = _u(index).reshape(-1).long()
    rows = torch.arange(stacked.shape[1], device=stacked.device)
    return _w(stacked[idx, rows])


@_export
def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):
    return _w(torch.addmm(_u(input), _u(x), _u(y), beta=beta, alpha=alpha))


@_export
def inner(x, y, name=None):
    return _w(torch.inner(_u(x), _u(y)))


@_export
def outer(x, y, name=None):
    return _w(torch.outer(_u(x).reshape(-1), _u(y).reshape(-1)))


@_export
def kron(x, y, name=None):
    return _w(torch.kron(_u(x), _u(y)))


@_export
def trace(x, offset=0, axis1=0, axis2=1, name=None):
    return _w(torch.diagonal(_u(x), offset, axis1, axis2).sum(-1))


@_export
def diagonal(x, offset=0, axis1=0, axis2=1, name=None):
    return _w(torch.diagonal(_u(x), offset, axis1, axis2))


@_export
def diff(x, n=1, axis=-1, prepend=None, append=None, name=None):
    return _w(torch.diff(_u(x), n, axis, _u(prepend), _u(append)))


@_export
def renorm(x, p, axis, max_norm):
    return _w(torch.renorm(_u(x), p, axis, max_norm))


@_export
def broadcast_shape(x_shape, y_shape):
    return list(torch.broadcast_shapes(tuple(x_shape), tuple(y_shape)))


# ----------------------------------------------------------------------------
# reductions
# ----------------------------------------------------------------------------
def _reduce_dim(axis, t):
    d = _axis(axis)
    if d is None:
        return None
    if isinstance(d, tuple) and len(d) == t.dim() and t.dim() > 0:
        return None if len(set(x % t.dim() for x in d)) == t.dim() else d
    return d


@_export
def sum(x, axis=None, dtype=None, keepdim=False, name=None):
    t = _u(x)
    dt = convert_dtype(dtype)
    if dt is None and (t.dtype == torch.bool or t.dtype == torch.int32):
        dt = torch.int64
    d = _reduce_dim(axis, t)
    if d is None:
        out = torch.sum(t, dtype=dt)
        if keepdim:
            out = out.reshape([1] * t.dim())
        return _w(out)
    return _w(torch.sum(t, dim=d, keepdim=keepdim, dtype=dt))


@_export
def nansum(x, axis=None, dtype=None, keepdim=False, name=None):
    t = _u(x)
    d = _reduce_dim(axis, t)
    dt = convert_dtype(dtype)
    if d is None:
        return _w(torch.nansum(t, dtype=dt))
    return _w(torch.nansum(t, dim=d, keepdim=keepdim, dtype=dt))


@_export
def mean(x, axis=None, keepdim=False, name=None):
    t = _u(x)
    d = _reduce_dim(axis, t)
    if d is None:
        out = torch.mean(t)
        if keepdim:
            out = out.reshape([1] * t.dim())
        return _w(out)
    return _w(torch.mean(t, dim=d, keepdim=keepdim))


@_export
def nanmean(x, axis=None, keepdim=False, name=None):
    t = _u(x)
    d = _reduce_dim(axis, t)
    if d is None:
        return _w(torch.nanmean(t))
    return _w(torch.nanmean(t, dim=d, keepdim=keepdim))


@_export
def prod(x, axis=None, keepdim=False, dtype=None, name=None):
    t = _u(x)
    dt = convert_dtype(dtype)
    d = _reduce_dim(axis, t)
    if d is None:
        out = torch.prod(t, dtype=dt)
        return _w(out.reshape([1] * t.dim()) if keepdim else out)
    if isinstance(d, tuple):
        out = t if dt is None else t.to(dt)
        for a in sorted((a % t.dim() for a in d), reverse=True):
            out = torch.prod(out, dim=a, keepdim=keepdim)
        return _w(out)
    return _w(torch.prod(t, dim=d, keepdim=keepdim, dtype=dt))


def _minmax(fn, x, axis, keepdim):
    t = _u(x)
    d = _reduce_dim(axis, t)
    if d is None:
        out = fn(t)
        return _w(out.reshape([1] * t.dim()) if keepdim else out)
    return _w(fn(t, dim=d, keepdim=keepdim))


@_export
def max(x, axis=None, keepdim=False, name=None):
    return _minmax(torch.amax, x, axis, keepdim)


@_export
def min(x, axis=None, keepdim=False, name=None):
    return _minmax(torch.amin, x, axis, keepdim)


@_export
def amax(x, axis=None, keepdim=False, name=None):
    return _minmax(torch.amax, x, axis, keepdim)


@_export
def amin(x, axis=None, keepdim=False, name=None):
    return _minmax(torch.amin, x, axis, keepdim)


@_export
def all(x, axis=None, keepdim=False, name=None):
    t = _u(x).bool()
    d = _reduce_dim(axis, t)
    if d is None:
        out = torch.all(t)
        return _w(out.reshape([1] * t.dim()) if keepdim else out)
    if isinstance(d, tuple):
        return _w(torch.all(t, dim=d, keepdim=keepdim)) if hasattr(torch, "all") else None
    return _w(torch.all(t, dim=d, keepdim=keepdim))


@_export
def any(x, axis=None, keepdim=False, name=None):
    t = _u(x).bool()
    d = _reduce_dim(axis, t)
    if d is None:
        out = torch.any(t)
        return _w(out.reshape([1] * t.dim()) if keepdim else out)
    return _w(torch.any(t, dim=d, keepdim=keepdim))


@_export
def logsumexp(x, axis=None, keepdim=False, name=None):
    t = _u(x)
    d = _reduce_dim(axis, t)
    if d is None:
        d = tuple(range(t.dim()))
    return _w(torch.logsumexp(t, dim=d, keepdim=keepdim))


@_export
def cumsum(x, axis=None, dtype=None, name=None):
    t = _u(x)
    if axis is None:
        t = t.reshape(-1)
        axis = 0
    return _w(torch.cumsum(t, int(axis), dtype=convert_dtype(dtype)))


@_export
def cumprod(x, dim=None, dtype=None, name=None):
    t = _u(x)
    if dim is None:
        t = t.reshape(-1)
        dim = 0
    return _w(torch.cumprod(t, int(dim), dtype=convert_dtype(dtype)))


@_export
def logcumsumexp(x, axis=None, dtype=None, name=None):
    t = _u(x)
    if dtype is not None:
        t = t.to(convert_dtype(dtype))
    if axis is None:
        t = t.reshape(-1)
        axis = 0
    return _w(torch.logcumsumexp(t, int(axis)))


@_export
def cummax(x, axis=None, dtype="int64", name=None):
    t = _u(x)
    if axis is None:
        t, axis = t.reshape(-1), 0
    v, i = torch.cummax(t, int(axis))
    return _w(v), _w(i.to(convert_dtype(dtype)))


@_export
def cummin(x, axis=None, dtype="int64", name=None):
    t = _u(x)
    if axis is None:
        t, axis = t.reshape(-1), 0
    v, i = torch.cummin(t, int(axis))
    return _w(v), _w(i.to(convert_dtype(dtype)))


@_export
def count_nonzero(x, axis=None, keepdim=False, name=None):
    t = _u(x)
    d = _reduce_dim(axis, t)
    out = torch.count_nonzero(t, dim=d)
    if keepdim and d is not None:
        for a in sorted([d] if isinstance(d, int) else list(d)):
            out = out.unsqueeze(a % t.dim())
    return _w(out)


# ----------------------------------------------------------------------------
# stat (reference: python/paddle/tensor/stat.py)
# ----------------------------------------------------------------------------
@_export
def var(x, axis=None, unbiased=True, keepdim=False, name=None):
    t = _u(x)
    d = _reduce_dim(axis, t)
    return _w(torch.var(t, dim=d, unbiased=unbiased, keepdim=keepdim))


@_export
def std(x, axis=None, unbiased=True, keepdim=False, name=None):
    t = _u(x)
    d = _reduce_dim(axis, t)
    return _w(torch.std(t, dim=d, unbiased=unbiased, keepdim=keepdim))


@_export
def median(x, axis=None, keepdim=False, name=None):
    t = _u(x)
    if axis is None:
        s = torch.sort(t.reshape(-1)).values
        n = s.numel()
        out = s[(n - 1) // 2] if n % 2 else (s[n // 2 - 1] + s[n // 2]) / 2
        if not t.is_floating_point():
            out = out.float()
        return _w(out.reshape([1] * t.dim()) if keepdim else out)
    s = torch.sort(t, dim=axis).values
    n = t.shape[axis]
    if n % 2:
        out = s.select(axis, (n - 1) // 2)
    else:
        out = (s.select(axis, n // 2 - 1) + s.select(axis, n // 2)) / 2
    if keepdim:
        out = out.unsqueeze(axis)
    return _w(out)


@_export
def nanmedian(x, axis=None, keepdim=True, name=None):
    """median ignoring NaNs; an even count averages the two middle values (reference
    python/paddle/tensor/stat.py nanmedian, phi nanmedian kernel), unlike torch.nanmedian's lower one"""
    t = _u(x)
    if axis is None:
        out = torch.nanquantile(t.reshape(-1), 0.5, interpolation="midpoint")
        return _w(out.reshape([1] * t.dim()) if keepdim else out.reshape([1]))
    axes = [axis] if isinstance(axis, int) else list(axis)
    axes = sorted(a % t.dim() for a in axes)
    keep = [d for d in range(t.dim()) if d not in axes]
    moved = t.permute(keep + axes).reshape([t.shape[d] for d in keep] + [-1])
    out = torch.nanquantile(moved, 0.5, dim=-1, interpolation="midpoint")
    if keepdim:
        out = out.reshape([1 if d in axes else t.shape[d] for d in range(t.dim())])
    return _w(out)


@_export
def quantile(x, q, axis=None, keepdim=False):
    t = _u(x)
    qq = torch.as_tensor(q, dtype=t.dtype, device=t.device)
    if axis is None:
        return _w(torch.quantile(t.reshape(-1), qq, keepdim=False))
    return _w(torch.quantile(t, qq, dim=axis, keepdim=keepdim))


@_export
def nanquantile(x, q, axis=None, keepdim=False):
    t = _u(x)
    qq = torch.as_tensor(q, dtype=t.dtype, device=t.device)
    if axis is None:
        return _w(torch.nanquantile(t.reshape(-1), qq))
    return _w(torch.nanquantile(t, qq, dim=axis, keepdim=keepdim))


@_export
def numel(x, name=None):
    return _w(torch.tensor(_u(x).numel(), dtype=torch.int64, device=_u(x).device))


# ----------------------------------------------------------------------------
# matmul family (reference: python/paddle/tensor/linalg.py:matmul)
# ----------------------------------------------------------------------------
@_export
def matmul(x, y, transpose_x=False, transpose_y=False, name=None):
    a = x._t if isinstance(x, Tensor) else torch.as_tensor(x)
    b = y._t if isinstance(y, Tensor) else torch.as_tensor(y)
    if a.is_cuda or b.is_cuda:   # GPU products: the own GEMM layouts (ops/gemm.py matmul)
        from ..ops import gemm as _gemm
        return _w(_gemm.matmul(a, b, transpose_x and a.dim() > 1, transpose_y and b.dim() > 1))
    if transpose_x:
        a = a.transpose(-1, -2) if a.dim() > 1 else a
    if transpose_y:
        b = b.transpose(-1, -2) if b.dim() > 1 else b
    return _w(torch.matmul(a, b))


@_export
def mm(input, mat2, name=None):
    a, b = _u(input), _u(mat2)
    if a.is_cuda:
        from ..ops import gemm as _gemm
        return _w(_gemm.matmul(a, b))
    return _w(torch.matmul(a, b))


@_export
def bmm(x, y, name=None):
    a, b = _u(x), _u(y)
    if a.is_cuda:
        from ..ops import gemm as _gemm
        return _w(_gemm.matmul(a, b))
    return _w(torch.bmm(a, b))


@_export
def mv(x, vec, name=None):
    return _w(torch.mv(_u(x), _u(vec)))


@_export
def dot(x, y, name=None):
    a, b = _u(x), _u(y)
    if a.dim() == 1:
        return _w(torch.dot(a, b))
    return _w((a * b).sum(-1))


register_ops(globals(), __all__)


def inverse(x, name=None):
    """(reference: tensor/math.py inverse) the matrix inverse over the last two axes"""
    from .. import linalg
    return linalg.inv(x)
