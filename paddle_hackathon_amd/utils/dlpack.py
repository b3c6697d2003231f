"""DLPack interop (reference: python/paddle/utils/dlpack.py). Zero-copy on HIP device memory."""
from __future__ import annotations

import torch.utils.dlpack as _dl

from ..framework.core import _wrap, Tensor

__all__ = ["to_dlpack", "from_dlpack"]


def to_dlpack(x):
    if not isinstance(x, Tensor):
        raise TypeError(f"The type of 'x' in to_dlpack must be paddle.Tensor, but received {type(x)}.")
    return _dl.to_dlpack(x._t.detach())


def from_dlpack(dlpack):
    return _wrap(_dl.from_dlpack(dlpack))
