"""Misc functionals: rnn helpers, distance (reference: python/paddle/nn/functional/*)."""
from __future__ import annotations

import torch

from ...framework.core import _wrap
from ...framework.dispatch import register_ops

_w = _wrap

__all__ = ["pairwise_distance"]


def pairwise_distance(x, y, p=2.0, epsilon=1e-6, keepdim=False, name=None):
    return _w(torch.nn.functional.pairwise_distance(x._t, y._t, p, epsilon, keepdim))


register_ops(globals(), __all__)
