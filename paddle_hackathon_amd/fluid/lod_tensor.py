"""``create_lod_tensor`` / ``create_random_int_lodtensor`` (reference:
python/paddle/fluid/lod_tensor.py)."""
from __future__ import annotations

import numpy as np

from . import core

__all__ = ["create_lod_tensor", "create_random_int_lodtensor"]


def create_lod_tensor(data, recursive_seq_lens, place=None):
    """``data``: numpy array, list of sequences (level-1 LoD inferred) or LoDTensor"""
    if isinstance(data, core.LoDTensor):
        return create_lod_tensor(np.asarray(data), recursive_seq_lens, place)
    if isinstance(data, list):
        lens = [len(seq) for seq in data]
        if [lens] != [list(l) for l in recursive_seq_lens][-1:]:
            raise ValueError("data and recursive_seq_lens do not match")
        arr = np.concatenate([np.asarray(s) for s in data]).reshape(-1, 1).astype("int64")
        return create_lod_tensor(arr, recursive_seq_lens, place)
    t = core.LoDTensor()
    t.set(np.asarray(data), place)
    t.set_recursive_sequence_lengths(recursive_seq_lens)
    if not t.has_valid_recursive_sequence_lengths():
        raise ValueError("the provided recursive_seq_lens info is invalid")
    return t


def create_random_int_lodtensor(recursive_seq_lens, base_shape, place, low, high):
    n = sum(recursive_seq_lens[-1])
    data = np.random.randint(low, high + 1, [n] + list(base_shape)).astype("int64")
    return create_lod_tensor(data, recursive_seq_lens, place)
