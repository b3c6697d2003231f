"""Tensor creation ops (reference: python/paddle/tensor/creation.py)."""
from __future__ import annotations

import numpy as np
import torch

from ..framework import core as _core
from ..framework.core import Tensor, to_tensor, _to_torch_device  # noqa: F401
from ..framework.dispatch import register_ops
from ._helpers import _u, _w, _int_list, _dtype_or_default, convert_dtype, default_device

__all__ = [
    "to_tensor", "zeros", "ones", "full", "empty", "zeros_like", "ones_like", "full_like",
    "empty_like", "arange", "linspace", "logspace", "eye", "diag", "diagflat", "tril", "triu",
    "meshgrid", "assign", "clone", "complex", "tril_indices", "triu_indices", "diag_embed",
    "create_parameter", "fill_constant",
]


def _shape(shape):
    if isinstance(shape, (int, np.integer)):
        return [int(shape)]
    return _int_list(shape)


def zeros(shape, dtype=None, name=None):
    return _w(torch.zeros(_shape(shape), dtype=_dtype_or_default(dtype), device=default_device()))


def ones(shape, dtype=None, name=None):
    return _w(torch.ones(_shape(shape), dtype=_dtype_or_default(dtype), device=default_device()))


def empty(shape, dtype=None, name=None):
    return _w(torch.empty(_shape(shape), dtype=_dtype_or_default(dtype), device=default_device()))


def full(shape, fill_value, dtype=None, name=None):
    if isinstance(fill_value, Tensor):
        fill_value = fill_value._t.item()
    if dtype is None:
        dt = torch.bool if isinstance(fill_value, bool) else _core._default_dtype
    else:
        dt = convert_dtype(dtype)
    return _w(torch.full(_shape(shape), fill_value, dtype=dt, device=default_device()))


def fill_constant(shape, dtype, value, force_cpu=False, out=None, name=None):
    t = full(shape, value, dtype)
    if out is not None:
        out._t = t._t
        return out
    return t


def _like(x, dtype):
    t = _u(x)
    return t, (t.dtype if dtype is None else convert_dtype(dtype))


def zeros_like(x, dtype=None, name=None):
    t, dt = _like(x, dtype)
    return _w(torch.zeros_like(t, dtype=dt))


def ones_like(x, dtype=None, name=None):
    t, dt = _like(x, dtype)
    return _w(torch.ones_like(t, dtype=dt))


def empty_like(x, dtype=None, name=None):
    t, dt = _like(x, dtype)
    return _w(torch.empty_like(t, dtype=dt))


def full_like(x, fill_value, dtype=None, name=None):
    t, dt = _like(x, dtype)
    if isinstance(fill_value, Tensor):
        fill_value = fill_value._t.item()
    return _w(torch.full_like(t, fill_value, dtype=dt))


def arange(start=0, end=None, step=1, dtype=None, name=None):
    start, end, step = (v._t.item() if isinstance(v, Tensor) else v for v in (start, end, step))
    if end is None:
        start, end = 0, start
    if dtype is None:
        dt = torch.int64 if all(isinstance(v, (int, np.integer)) for v in (start, end, step)) else _core._default_dtype
    else:
        dt = convert_dtype(dtype)
    return _w(torch.arange(start, end, step, dtype=dt, device=default_device()))


def linspace(start, stop, num, dtype=None, name=None):
    start, stop, num = (v._t.item() if isinstance(v, Tensor) else v for v in (start, stop, num))
    dt = _dtype_or_default(dtype)
    return _w(torch.linspace(start, stop, int(num), dtype=torch.float64, device=default_device()).to(dt))


def logspace(start, stop, num, base=10.0, dtype=None, name=None):
    start, stop, num, base = (v._t.item() if isinstance(v, Tensor) else v for v in (start, stop, num, base))
    dt = _dtype_or_default(dtype)
    return _w(torch.logspace(start, stop, int(num), base=base, dtype=torch.float64, device=default_device()).to(dt))


def eye(num_rows, num_columns=None, dtype=None, name=None):
    num_columns = num_rows if num_columns is None else num_columns
    return _w(torch.eye(int(num_rows), int(num_columns), dtype=_dtype_or_default(dtype), device=default_device()))


def diag(x, offset=0, padding_value=0, name=None):
    t = _u(x)
    if t.dim() == 1 and padding_value != 0:
        n = t.shape[0] + abs(offset)
        out = torch.full((n, n), padding_value, dtype=t.dtype, device=t.device)
        out = out + torch.diag(t, offset) - torch.diag(torch.full_like(t, padding_value), offset)
        return _w(out)
    return _w(torch.diag(t, offset))


def diagflat(x, offset=0, name=None):
    return _w(torch.diagflat(_u(x), offset))


def diag_embed(input, offset=0, dim1=-2, dim2=-1):
    return _w(torch.diag_embed(_u(input), offset, dim1, dim2))


def tril(x, diagonal=0, name=None):
    return _w(torch.tril(_u(x), diagonal))


def triu(x, diagonal=0, name=None):
    return _w(torch.triu(_u(x), diagonal))


def tril_indices(row, col, offset=0, dtype="int64"):
    return _w(torch.tril_indices(row, col, offset, dtype=convert_dtype(dtype), device=default_device()))


def triu_indices(row, col=None, offset=0, dtype="int64"):
    col = row if col is None else col
    return _w(torch.triu_indices(row, col, offset, dtype=convert_dtype(dtype), device=default_device()))


def meshgrid(*args, **kwargs):
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = args[0]
    return [_w(t) for t in torch.meshgrid(*[_u(a) for a in args], indexing="ij")]


def assign(x, output=None):
    if isinstance(x, Tensor):
        t = x._t.clone()
    else:
        t = _core._to_torch(np.asarray(x) if not isinstance(x, (int, float)) else x)
        if t.dtype == torch.float64 and not isinstance(x, np.ndarray):
            t = t.float()
    if output is not None:
        with torch.no_grad():
            if output._t.shape == t.shape:
                output._t.copy_(t)
            else:
                output._t = t
        return output
    return _w(t)


def clone(x, name=None):
    return _w(_u(x).clone())


def complex(real, imag, name=None):
    return _w(torch.complex(_u(real), _u(imag)))


def create_parameter(shape, dtype, name=None, attr=None, is_bias=False, default_initializer=None):
    from ..nn.layer.layers import _create_parameter
    return _create_parameter(shape, dtype, attr, is_bias, default_initializer, name=name)


register_ops(globals(), [n for n in __all__ if n not in ("create_parameter",)])
