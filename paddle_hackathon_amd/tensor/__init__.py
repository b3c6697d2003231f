"""``paddle.tensor``: op modules + Tensor method/operator patching
(reference: python/paddle/tensor/__init__.py:tensor_method_func,
python/paddle/fluid/dygraph/math_op_patch.py)."""
from __future__ import annotations

import numpy as np
import torch

from ..framework.core import Tensor, Parameter, _wrap, _unwrap
from ..framework.dispatch import register_ops
from . import creation, math, manipulation, logic, search, random, linalg, attribute  # noqa: F401
from .creation import *  # noqa: F401,F403
from .math import *  # noqa: F401,F403
from .manipulation import *  # noqa: F401,F403
from .logic import *  # noqa: F401,F403
from .search import *  # noqa: F401,F403
from .random import *  # noqa: F401,F403
from .linalg import *  # noqa: F401,F403
from .attribute import *  # noqa: F401,F403


# ----------------------------------------------------------------------------
# indexing ops (recorded in static mode like any other op)
# ----------------------------------------------------------------------------
def _index(idx):
    if isinstance(idx, Tensor):
        t = idx._t
        return t if t.dtype == torch.bool else t.long()
    if isinstance(idx, tuple):
        return tuple(_index(i) for i in idx)
    if isinstance(idx, list):
        if any(isinstance(i, (Tensor, list, slice, tuple)) or i is None or i is Ellipsis for i in idx):
            return tuple(_index(i) for i in idx)
        return torch.as_tensor(idx)
    if isinstance(idx, np.ndarray):
        return torch.from_numpy(idx)
    return idx


def getitem(x, idx):
    t = x._t
    if t.dim() == 0 and idx is not Ellipsis and idx != ():   # 0-d reads as shape [1] (no 0-d tensors in the reference)
        t = t.reshape(1)
    if isinstance(idx, Tensor) and idx._t.numel() == 1 and idx._t.dim() <= 1 and not idx._t.is_floating_point() \
            and idx._t.dtype != torch.bool:
        # scalar tensor index (e.g. a traced loop counter): a gather, so the shape is data-independent
        i = idx._t.reshape(1).to(torch.int64)
        i = torch.where(i < 0, i + t.shape[0], i)
        return _wrap(torch.index_select(t, 0, i.to(t.device)).squeeze(0))
    items = idx if isinstance(idx, tuple) else (idx,)
    import builtins
    if builtins.any(isinstance(i, builtins.slice) and isinstance(i.step, int) and i.step < 0 for i in items):
        return _wrap(_neg_step_getitem(t, items))
    return _wrap(t[_index(idx)])


def _neg_step_getitem(t, items):
    """basic indexing with negative slice steps (x[::-1], x[5:1:-2]; torch has no negative
    strides): the negative-step slices are taken as full dims, then gathered by index_select
    (differentiable) with Python's slice arithmetic"""
    import builtins
    if builtins.any(i is Ellipsis for i in items):
        k = list(items).index(Ellipsis)
        n_real = builtins.sum(1 for i in items if i is not None and i is not Ellipsis)
        items = items[:k] + (builtins.slice(None),) * (t.dim() - n_real) + items[k + 1:]
    first, picks, out_dim, in_dim = [], [], 0, 0
    for it in items:
        if it is None:
            first.append(None)
            out_dim += 1
        elif isinstance(it, builtins.slice) and it.step is not None and it.step < 0:
            first.append(builtins.slice(None))
            idx = builtins.range(*it.indices(t.shape[in_dim]))
            picks.append((out_dim, torch.tensor(list(idx), dtype=torch.long, device=t.device)))
            out_dim += 1
            in_dim += 1
        elif isinstance(it, builtins.slice):
            first.append(it)
            out_dim += 1
            in_dim += 1
        else:
            first.append(_index(it))
            in_dim += 1
            if not isinstance(it, int):
                out_dim += 1
    out = t[tuple(first)]
    for d, ix in picks:
        out = torch.index_select(out, d, ix)
    return out


def setitem(x, idx, value):
    v = value._t if isinstance(value, Tensor) else value
    if isinstance(v, np.ndarray):
        v = torch.from_numpy(v)
    if isinstance(v, torch.Tensor) and v.device != x._t.device:
        v = v.to(x._t.device)
    if x._t.is_leaf and x._t.requires_grad:
        with torch.no_grad():
            x._t[_index(idx)] = v
    else:
        x._t[_index(idx)] = v
    return x


_ns = {"getitem": getitem, "setitem": setitem}
register_ops(_ns, ["getitem", "setitem"])
getitem = _ns["getitem"]
setitem = _ns["setitem"]


# ----------------------------------------------------------------------------
# method patching
# ----------------------------------------------------------------------------
_METHODS = [
    "matmul", "dot", "cov", "corrcoef", "norm", "cond", "transpose", "lstsq", "dist", "t",
    "cross", "cholesky", "bmm", "histogram", "bincount", "mv", "matrix_power", "qr", "eigvals",
    "eigvalsh", "abs", "acos", "all", "any", "asin", "atan", "ceil", "ceil_", "cos", "cosh",
    "cumsum", "cumprod", "logcumsumexp", "logit", "exp", "exp_", "floor", "floor_", "increment",
    "log", "log2", "log10", "logsumexp", "multiplex", "pow", "prod", "reciprocal", "reciprocal_",
    "round", "round_", "rsqrt", "rsqrt_", "scale", "scale_", "sign", "sin", "sinh", "sqrt",
    "sqrt_", "square", "stanh", "sum", "nansum", "nanmean", "tanh", "tanh_", "add_n", "max",
    "amax", "maximum", "min", "amin", "minimum", "fmax", "fmin", "mm", "inner", "outer",
    "divide", "floor_divide", "remainder", "mod", "floor_mod", "multiply", "add", "add_",
    "subtract", "subtract_", "inverse", "log1p", "erf", "addmm", "clip", "clip_", "trace",
    "kron", "kthvalue", "isfinite", "isinf", "isnan", "broadcast_shape", "conj", "neg", "lgamma",
    "equal", "equal_all", "greater_equal", "greater_than", "is_empty", "less_equal", "less_than",
    "logical_and", "logical_not", "logical_or", "logical_xor", "not_equal", "allclose",
    "isclose", "is_tensor", "concat", "expand", "broadcast_to", "expand_as", "flatten",
    "flatten_", "gather", "gather_nd", "reshape", "reshape_", "reverse", "scatter", "scatter_",
    "scatter_nd_add", "scatter_nd", "shard_index", "slice", "split", "chunk", "tensordot",
    "squeeze", "squeeze_", "stack", "strided_slice", "unique", "unique_consecutive",
    "unsqueeze", "unsqueeze_", "unstack", "flip", "rot90", "unbind", "roll", "tile", "argmax",
    "argmin", "argsort", "masked_select", "topk", "where", "index_select", "nonzero", "sort",
    "index_sample", "mean", "std", "var", "numel", "median", "nanmedian", "quantile",
    "nanquantile", "is_complex", "is_integer", "rank", "real", "imag", "is_floating_point",
    "digamma", "diagonal", "trunc", "frac", "bitwise_and", "bitwise_or", "bitwise_xor",
    "bitwise_not", "broadcast_tensors", "eig", "uniform_", "multi_dot", "solve",
    "cholesky_solve", "triangular_solve", "asinh", "atanh", "acosh", "lu", "lu_unpack",
    "as_complex", "as_real", "rad2deg", "deg2rad", "gcd", "lcm", "diff", "mode", "lerp",
    "lerp_", "erfinv", "erfinv_", "angle", "moveaxis", "repeat_interleave", "take_along_axis",
    "put_along_axis", "put_along_axis_", "exponential_", "heaviside",
    # extras commonly used on paddle Tensors
    "sigmoid", "tan", "expm1", "masked_fill", "fill_", "zero_", "fill_diagonal_", "view",
    "view_as", "normal_", "multiply_", "divide_", "square_", "abs_", "neg_", "sin_", "cos_",
    "log_", "sigmoid_", "index_add", "index_put", "count_nonzero", "unfold", "cummax",
    "cummin", "nan_to_num", "atleast_1d", "atleast_2d", "atleast_3d", "det", "slogdet", "pinv",
    "inv", "svd", "matrix_rank", "vector_norm", "amax", "searchsorted", "bucketize",
]


def _patch():
    g = globals()
    for n in _METHODS:
        f = g.get(n)
        if f is None:
            continue
        if n in ("shape",):
            continue
        setattr(Tensor, n, f)

    def _r(f):
        return lambda self, other: f(other, self)

    ops = {
        "__add__": g["add"], "__radd__": _r(g["add"]),
        "__sub__": g["subtract"], "__rsub__": _r(g["subtract"]),
        "__mul__": g["multiply"], "__rmul__": _r(g["multiply"]),
        "__truediv__": g["divide"], "__rtruediv__": _r(g["divide"]),
        "__div__": g["divide"], "__rdiv__": _r(g["divide"]),
        "__floordiv__": g["floor_divide"], "__rfloordiv__": _r(g["floor_divide"]),
        "__mod__": g["remainder"], "__rmod__": _r(g["remainder"]),
        "__pow__": g["pow"], "__rpow__": _r(g["pow"]),
        "__matmul__": g["matmul"], "__rmatmul__": _r(g["matmul"]),
        "__eq__": g["equal"], "__ne__": g["not_equal"],
        "__lt__": g["less_than"], "__le__": g["less_equal"],
        "__gt__": g["greater_than"], "__ge__": g["greater_equal"],
        "__and__": g["bitwise_and"], "__or__": g["bitwise_or"], "__xor__": g["bitwise_xor"],
        "__rand__": _r(g["bitwise_and"]), "__ror__": _r(g["bitwise_or"]), "__rxor__": _r(g["bitwise_xor"]),
        "__getitem__": getitem, "__setitem__": setitem,
    }
    for k, f in ops.items():
        setattr(Tensor, k, f)
    Tensor.__neg__ = lambda self: g["neg"](self)
    Tensor.__abs__ = lambda self: g["abs"](self)
    Tensor.__invert__ = lambda self: g["bitwise_not"](self) if self._t.dtype != torch.bool else g["logical_not"](self)
    Tensor.__pos__ = lambda self: self

    def _iop(tname):
        def f(self, other):
            o = other._t if isinstance(other, Tensor) else other
            if self._t.requires_grad and self._t.is_leaf:
                # paddle semantics: `x += y` on a leaf that needs grad rebinds the handle
                self._t = getattr(torch, tname)(self._t, o)
            else:
                getattr(self._t, tname + "_")(o)
            return self
        return f

    Tensor.__iadd__ = _iop("add")
    Tensor.__isub__ = _iop("sub")
    Tensor.__imul__ = _iop("mul")
    Tensor.__itruediv__ = _iop("div")


_patch()


def __getattr__(name):   # tensor arrays (their module imports fluid, which imports this package)
    if name in ("create_array", "array_write", "array_read", "array_length"):
        from . import array as _a
        return getattr(_a, name)
    if name in ("stat", "array"):
        import importlib
        return importlib.import_module("." + name, __name__)
    raise AttributeError(name)
