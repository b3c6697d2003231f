"""Search / sort ops (reference: python/paddle/tensor/search.py)."""
from __future__ import annotations

import torch

from ..framework.core import Tensor, convert_dtype
from ..framework.dispatch import register_ops
from ._helpers import _u, _w

__all__ = ["argmax", "argmin", "argsort", "sort", "topk", "kthvalue", "mode", "searchsorted",
           "bucketize", "msort"]


def argmax(x, axis=None, keepdim=False, dtype="int64", name=None):
    t = _u(x)
    if axis is None:
        out = torch.argmax(t.reshape(-1))
        if keepdim:
            out = out.reshape([1] * t.dim())
    else:
        out = torch.argmax(t, dim=int(axis), keepdim=keepdim)
    return _w(out.to(convert_dtype(dtype)))


def argmin(x, axis=None, keepdim=False, dtype="int64", name=None):
    t = _u(x)
    if axis is None:
        out = torch.argmin(t.reshape(-1))
        if keepdim:
            out = out.reshape([1] * t.dim())
    else:
        out = torch.argmin(t, dim=int(axis), keepdim=keepdim)
    return _w(out.to(convert_dtype(dtype)))


def argsort(x, axis=-1, descending=False, name=None):
    return _w(torch.argsort(_u(x), dim=axis, descending=descending, stable=True))


def sort(x, axis=-1, descending=False, name=None):
    return _w(torch.sort(_u(x), dim=axis, descending=descending, stable=True).values)


def msort(x, name=None):
    return sort(x, 0)


def topk(x, k, axis=None, largest=True, sorted=True, name=None):
    if isinstance(k, Tensor):
        k = int(k._t.item())
    axis = -1 if axis is None else axis
    v, i = torch.topk(_u(x), k, dim=axis, largest=largest, sorted=sorted)
    return _w(v), _w(i)


def kthvalue(x, k, axis=None, keepdim=False, name=None):
    axis = -1 if axis is None else axis
    v, i = torch.kthvalue(_u(x), k, dim=axis, keepdim=keepdim)
    return _w(v), _w(i)


def mode(x, axis=-1, keepdim=False, name=None):
    v, i = torch.mode(_u(x), dim=axis, keepdim=keepdim)
    return _w(v), _w(i)


def searchsorted(sorted_sequence, values, out_int32=False, right=False, name=None):
    return _w(torch.searchsorted(_u(sorted_sequence), _u(values), out_int32=out_int32, right=right))


def bucketize(x, sorted_sequence, out_int32=False, right=False, name=None):
    return _w(torch.bucketize(_u(x), _u(sorted_sequence), out_int32=out_int32, right=right))


register_ops(globals(), __all__)
