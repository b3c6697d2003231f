"""Misc functionals: rnn helpers, distance (reference: python/paddle/nn/functional/*)."""
from __future__ import annotations

import torch

from ...framework.core import _wrap
from ...framework.dispatch import register_ops

_w = _wrap

__all__ = ["pairwise_distance"]


def pairwise_distance(x, y, p=2.0, epsilon=1e-6, keepdim=False, name=None):
    """p-norm of x - y along axis 1 (reference nn/layer/distance.py: p_norm(x - y, p, axis=1); the
    oracle is np.linalg.norm(x - y, ord=p, axis=1) — epsilon is not added to the difference)"""
    d = x._t - y._t
    return _w(torch.linalg.vector_norm(d, ord=p, dim=1 if d.dim() > 1 else 0, keepdim=keepdim))


register_ops(globals(), __all__)
