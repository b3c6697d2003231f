"""``fluid.input`` (reference: python/paddle/fluid/input.py): the v2 one_hot / embedding, which
append the new dimension instead of consuming a trailing 1."""
from __future__ import annotations

import torch.nn.functional as TF

from .layers._common import T, W

__all__ = ["one_hot", "embedding"]


def one_hot(input, depth, allow_out_of_range=False):
    ids = T(input).long()
    valid = (ids >= 0) & (ids < depth)
    if not allow_out_of_range and not bool(valid.all()):
        raise ValueError("one_hot: index out of range [0, depth)")
    return W(TF.one_hot(ids.clamp(0, depth - 1), depth).float() * valid[..., None].float())


def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None, param_attr=None,
              dtype="float32"):
    from ..nn.layer.layers import _create_parameter
    from ..nn import initializer as I
    w = _create_parameter(list(size), dtype, param_attr, default_initializer=I.XavierUniform())
    if padding_idx is not None and padding_idx < 0:
        padding_idx += size[0]
    return W(TF.embedding(T(input).long(), T(w), padding_idx=padding_idx))
