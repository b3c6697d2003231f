"""Shared helpers for the tensor op modules."""
from __future__ import annotations

import numpy as np
import torch

from ..framework.core import Tensor, _wrap, _unwrap, convert_dtype, default_device, _default_dtype  # noqa: F401
from ..framework import core as _core

_u = _unwrap
_w = _wrap


def _int_list(v):
    """Normalise a paddle shape/axes argument (int, list of int/Tensor, Tensor) to list[int]."""
    if v is None:
        return None
    if isinstance(v, Tensor):
        return [int(a) for a in v._t.reshape(-1).tolist()]
    if isinstance(v, torch.Tensor):
        return [int(a) for a in v.reshape(-1).tolist()]
    if isinstance(v, (int, np.integer)):
        return [int(v)]
    out = []
    for a in v:
        if isinstance(a, Tensor):
            out.append(int(a._t.item()))
        else:
            out.append(int(a))
    return out


def _axis(axis):
    """paddle axis (None | int | list | Tensor) -> torch dim (None | int | tuple)."""
    if axis is None:
        return None
    if isinstance(axis, (int, np.integer)):
        return int(axis)
    if isinstance(axis, Tensor):
        axis = axis._t.reshape(-1).tolist()
        return int(axis[0]) if len(axis) == 1 else tuple(int(a) for a in axis)
    axis = [int(a) if not isinstance(a, Tensor) else int(a._t.item()) for a in axis]
    if len(axis) == 0:
        return None
    return tuple(axis)


def _scalar(v):
    if isinstance(v, Tensor):
        return v._t.item() if v._t.numel() == 1 else v._t
    return v


def _to_t(x, like=None):
    """Anything -> torch tensor (python scalars stay scalars for torch broadcasting)."""
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, np.ndarray):
        t = torch.from_numpy(x)
        return t.to(like.device) if like is not None else t.to(default_device())
    return x


def _dev(device=None):
    return default_device() if device is None else device


def _dtype_or_default(dtype):
    d = convert_dtype(dtype)
    return _core._default_dtype if d is None else d
