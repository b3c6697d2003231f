"""paddle.incubate.multiprocessing (reference: python/paddle/incubate/multiprocessing/
{__init__,reductions}.py): the stdlib ``multiprocessing`` API plus pickling reductions that
share framework Tensors between processes without copying (CPU tensors through shared
memory, HIP tensors through IPC handles — torch.multiprocessing's reductions)."""
from __future__ import annotations

import multiprocessing
from multiprocessing import *  # noqa: F401,F403

import torch.multiprocessing as _tmp  # noqa: F401  (registers torch.Tensor reductions)
from multiprocessing.reduction import ForkingPickler

from ..framework.core import Tensor, Parameter, _wrap

__all__ = list(getattr(multiprocessing, "__all__", []))


def _rebuild(t, stop_gradient, name):
    out = _wrap(t)
    out.stop_gradient = stop_gradient
    out.name = name
    return out


def _reduce_tensor(x):
    t = x._t.detach()
    if not t.is_cuda:
        t = t.share_memory_()
    return _rebuild, (t, x.stop_gradient, x.name)


def init_reductions():
    ForkingPickler.register(Tensor, _reduce_tensor)
    ForkingPickler.register(Parameter, _reduce_tensor)


init_reductions()
