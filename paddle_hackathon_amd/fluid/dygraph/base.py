"""``fluid.dygraph.base`` (reference: python/paddle/fluid/dygraph/base.py): mode switches and
``to_variable``."""
from __future__ import annotations

import contextlib

import numpy as np

from ...framework import core as _core
from ...autograd import no_grad as _no_grad, grad  # noqa: F401
from ..core import LoDTensor

__all__ = ["no_grad", "no_grad_", "grad", "guard", "enable_dygraph", "disable_dygraph", "enabled", "to_variable"]

no_grad = _no_grad
no_grad_ = _no_grad


def enabled():
    return _core.in_dynamic_mode()


def enable_dygraph(place=None):
    from ... import disable_static
    disable_static(place)


def disable_dygraph():
    from ... import enable_static
    enable_static()


@contextlib.contextmanager
def guard(place=None):
    """run the block in dygraph mode (on ``place``)"""
    prev = _core._mode.static
    _core._mode.static = False
    prev_dev = None
    if place is not None:
        prev_dev = _core.get_device()
        _core.set_device(place)
    try:
        yield
    finally:
        _core._mode.static = prev
        if prev_dev is not None:
            _core.set_device(prev_dev)


def to_variable(value, name=None, zero_copy=None, dtype=None):
    """numpy array / LoDTensor / Tensor / list -> dygraph Tensor (LoD kept)"""
    if isinstance(value, _core.Tensor) and not isinstance(value, LoDTensor):
        return value
    lod = getattr(value, "_lod", None)
    arr = np.asarray(value) if not isinstance(value, _core.Tensor) else value.numpy()
    t = _core.to_tensor(arr, dtype=dtype)
    if lod:
        t._lod = lod
    if name:
        t.name = name
    return t
