"""Tensor attribute queries + einsum (reference: python/paddle/tensor/attribute.py, einsum.py)."""
from __future__ import annotations

import torch

from ..framework.core import Tensor
from ..framework.dispatch import register_ops
from ._helpers import _u, _w

__all__ = ["shape", "rank", "is_complex", "is_integer", "is_floating_point", "einsum"]


def shape(input):
    t = _u(input)
    return _w(torch.tensor(list(t.shape), dtype=torch.int32, device=t.device))


def rank(input):
    t = _u(input)
    return _w(torch.tensor(t.dim(), dtype=torch.int32, device=t.device))


def is_complex(x):
    return _u(x).is_complex()


def is_integer(x):
    t = _u(x)
    return not (t.is_floating_point() or t.is_complex() or t.dtype == torch.bool)


def is_floating_point(x):
    return _u(x).is_floating_point()


def einsum(equation, *operands):
    if len(operands) == 1 and isinstance(operands[0], (list, tuple)):
        operands = operands[0]
    return _w(torch.einsum(equation, *[_u(o) for o in operands]))


register_ops(globals(), ["shape", "rank", "einsum"])
