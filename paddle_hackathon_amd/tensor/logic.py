"""Comparison / logical / bitwise ops (reference: python/paddle/tensor/logic.py)."""
from __future__ import annotations

import torch

from ..framework.core import Tensor, is_tensor
from ..framework.dispatch import register_ops
from ._helpers import _u, _w
from .math import _bin

__all__ = [
    "equal", "equal_all", "greater_equal", "greater_than", "is_empty", "less_equal", "less_than",
    "logical_and", "logical_not", "logical_or", "logical_xor", "bitwise_and", "bitwise_not",
    "bitwise_or", "bitwise_xor", "not_equal", "allclose", "isclose", "is_tensor",
]


def _cmp(f):
    def op(x, y, name=None):
        a, b = _bin(x, y)
        return _w(f(a, b))
    op.__name__ = f.__name__
    return op


equal = _cmp(torch.eq)
not_equal = _cmp(torch.ne)
greater_equal = _cmp(torch.ge)
greater_than = _cmp(torch.gt)
less_equal = _cmp(torch.le)
less_than = _cmp(torch.lt)
for _n in ("equal", "not_equal", "greater_equal", "greater_than", "less_equal", "less_than"):
    globals()[_n].__name__ = _n


def equal_all(x, y, name=None):
    a, b = _u(x), _u(y)
    return _w(torch.tensor(a.shape == b.shape and bool(torch.equal(a, b)), device=a.device))


def is_empty(x, name=None):
    return _w(torch.tensor(_u(x).numel() == 0, device=_u(x).device))


def _logic(f):
    def op(x, y=None, out=None, name=None):
        a, b = _bin(x, y)
        r = f(a, b)
        if out is not None:
            out._t = r
            return out
        return _w(r)
    return op


logical_and = _logic(torch.logical_and)
logical_or = _logic(torch.logical_or)
logical_xor = _logic(torch.logical_xor)
bitwise_and = _logic(torch.bitwise_and)
bitwise_or = _logic(torch.bitwise_or)
bitwise_xor = _logic(torch.bitwise_xor)
for _n in ("logical_and", "logical_or", "logical_xor", "bitwise_and", "bitwise_or", "bitwise_xor"):
    globals()[_n].__name__ = _n


def logical_not(x, out=None, name=None):
    return _w(torch.logical_not(_u(x)))


def bitwise_not(x, out=None, name=None):
    return _w(torch.bitwise_not(_u(x)))


def allclose(x, y, rtol=1e-05, atol=1e-08, equal_nan=False, name=None):
    a, b = _u(x), _u(y)
    return _w(torch.tensor(torch.allclose(a, b, rtol, atol, equal_nan), device=a.device))


def isclose(x, y, rtol=1e-05, atol=1e-08, equal_nan=False, name=None):
    return _w(torch.isclose(_u(x), _u(y), rtol, atol, equal_nan))


register_ops(globals(), [n for n in __all__ if n != "is_tensor"])
