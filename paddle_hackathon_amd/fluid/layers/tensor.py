"""``fluid.layers`` tensor creation / conversion functions (reference:
python/paddle/fluid/layers/tensor.py)."""
from __future__ import annotations

import numpy as np
import torch

from ...framework.core import Tensor
from ._common import T, W, dt, dev, write_to, register, static_mode, static_source

__all__ = ["create_tensor", "create_parameter", "create_global_var", "cast", "tensor_array_to_tensor", "concat",
           "sums", "assign", "fill_constant_batch_size_like", "fill_constant", "argmin", "argmax", "argsort", "ones",
           "zeros", "reverse", "has_inf", "has_nan", "isfinite", "range", "linspace", "zeros_like", "ones_like",
           "diag", "eye", "triu"]

_BUILDERS = {"create_tensor", "create_parameter", "create_global_var", "assign", "fill_constant", "ones", "zeros",
             "range", "linspace", "eye", "sums", "tensor_array_to_tensor", "concat", "zeros_like", "ones_like"}


def create_tensor(dtype, name=None, persistable=False):
    t = W(torch.empty(0, dtype=dt(dtype), device=dev()))
    t.persistable = persistable
    if name:
        t.name = name
    return t


def create_parameter(shape, dtype, name=None, attr=None, is_bias=False, default_initializer=None):
    from ... import static
    return static.create_parameter(shape, dtype, name, attr, is_bias, default_initializer)


def create_global_var(shape, value, dtype, persistable=False, force_cpu=False, name=None):
    from ... import static
    return static.create_global_var(shape, value, dtype, persistable, force_cpu, name)


def cast(x, dtype):
    return W(T(x).to(dt(dtype)), x)


def _shape_list(shape):
    if isinstance(shape, Tensor):
        return [int(v) for v in T(shape).tolist()]
    return [int(T(s).item()) if isinstance(s, Tensor) else int(s) for s in shape]


def concat(input, axis=0, name=None):
    from ...tensor import concat as _concat
    xs = list(input) if isinstance(input, (list, tuple)) else [input]
    a = int(T(axis).item()) if isinstance(axis, Tensor) else axis
    return _concat(xs, a)


def tensor_array_to_tensor(input, axis=1, name=None, use_stack=False):
    """-> (concat / stack of the array's tensors along ``axis``, int32 sizes along ``axis``)"""
    from ...tensor import concat as _concat, stack as _stack
    xs = list(input)
    out = _stack(xs, axis) if use_stack else _concat(xs, axis)
    sizes = [1 if use_stack else T(x).shape[axis] for x in xs]
    return out, W(torch.tensor(sizes, dtype=torch.int32, device=dev()))


def sums(input, out=None):
    from ...tensor import add_n
    r = add_n(list(input))
    return write_to(out, r) if out is not None else r


def assign(input, output=None):
    from ...tensor import assign as _assign
    if isinstance(input, (np.ndarray, list, tuple, float, int, bool)):
        arr = np.asarray(input)
        r = _const(lambda: W(torch.as_tensor(arr, device=dev())), "assign_value")
        return write_to(output, r) if output is not None else r
    r = _assign(input)
    return write_to(output, r) if output is not None else r


def _const(fn, name):
    """eager value, or in static mode a recorded source op producing it every run"""
    with _eager():
        val = fn()
    if static_mode():
        return static_source(fn, name, T(val))
    return val


class _eager:
    def __enter__(self):
        from ...framework import core as _c
        self.prev = _c._mode.static
        _c._mode.static = False

    def __exit__(self, *a):
        from ...framework import core as _c
        _c._mode.static = self.prev


def fill_constant(shape, dtype, value, force_cpu=False, out=None, name=None):
    from ...tensor import full
    if isinstance(value, Tensor) and not static_mode():
        value = T(value).item()
    shp, d = _shape_list(shape), dt(dtype)
    r = _const(lambda: full(shp, value, d), "fill_constant")
    return write_to(out, r) if out is not None else r


def fill_constant_batch_size_like(input, shape, dtype, value, input_dim_idx=0, output_dim_idx=0, force_cpu=False):
    shp = list(shape)
    shp[output_dim_idx] = T(input).shape[input_dim_idx]
    return W(torch.full(shp, value, dtype=dt(dtype), device=dev()))


def argmin(x, axis=0):
    return W(T(x).argmin(axis))


def argmax(x, axis=0):
    return W(T(x).argmax(axis))


def argsort(input, axis=-1, descending=False, name=None):
    v, i = torch.sort(T(input), dim=axis, descending=descending, stable=True)
    return W(v), W(i)


def ones(shape, dtype, force_cpu=False):
    return fill_constant(shape, dtype, 1.0)


def zeros(shape, dtype, force_cpu=False, name=None):
    return fill_constant(shape, dtype, 0.0)


def reverse(x, axis):
    axes = [axis] if isinstance(axis, int) else list(axis)
    return W(torch.flip(T(x), axes))


def has_inf(x):
    return W(torch.isinf(T(x)).any().reshape(1))


def has_nan(x):
    return W(torch.isnan(T(x)).any().reshape(1))


def isfinite(x):
    return W(torch.isfinite(T(x)).all().reshape(1))


def range(start, end, step, dtype, name=None):
    from ...tensor import arange
    v = lambda a: T(a).item() if isinstance(a, Tensor) else a  # noqa: E731
    return arange(v(start), v(end), v(step), dt(dtype))


def linspace(start, stop, num, dtype=None, name=None):
    from ...tensor import linspace as _lin
    v = lambda a: T(a).item() if isinstance(a, Tensor) else a  # noqa: E731
    return _lin(v(start), v(stop), int(v(num)), dt(dtype or "float32"))


def zeros_like(x, out=None):
    from ...tensor import zeros_like as _zl
    r = _zl(x)
    return write_to(out, r) if out is not None else r


def ones_like(x, out=None):
    from ...tensor import ones_like as _ol
    r = _ol(x)
    return write_to(out, r) if out is not None else r


def diag(diagonal):
    d = T(diagonal) if isinstance(diagonal, Tensor) else torch.as_tensor(np.asarray(diagonal), device=dev())
    return W(torch.diag(d))


def eye(num_rows, num_columns=None, batch_shape=None, dtype="float32", name=None):
    from ...tensor import eye as _eye
    out = _eye(num_rows, num_columns, dt(dtype))
    if batch_shape:
        out = W(T(out).expand(list(batch_shape) + list(T(out).shape)).clone())
    return out


def triu(x, diagonal=0, name=None):
    return W(torch.triu(T(x), diagonal))


register(globals(), __all__, skip=_BUILDERS)
