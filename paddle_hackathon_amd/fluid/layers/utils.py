"""``fluid.layers.utils`` (reference: python/paddle/fluid/layers/utils.py): nested-structure
helpers used by control flow and RNN code."""
from __future__ import annotations

import collections.abc

__all__ = ["flatten", "pack_sequence_as", "map_structure", "is_sequence", "assert_same_structure",
           "convert_to_list"]


def is_sequence(seq):
    if isinstance(seq, dict):
        return True
    return isinstance(seq, collections.abc.Sequence) and not isinstance(seq, str)


def _sorted(d):
    return [d[k] for k in sorted(d)]


def flatten(nest):
    if not is_sequence(nest):
        return [nest]
    items = _sorted(nest) if isinstance(nest, dict) else list(nest)
    out = []
    for v in items:
        out.extend(flatten(v))
    return out


def _pack(structure, flat, index):
    if not is_sequence(structure):
        return flat[index], index + 1
    if isinstance(structure, dict):
        res = {}
        for k in sorted(structure):
            res[k], index = _pack(structure[k], flat, index)
        return res, index
    vals = []
    for v in structure:
        p, index = _pack(v, flat, index)
        vals.append(p)
    if isinstance(structure, tuple) and hasattr(structure, "_fields"):
        return type(structure)(*vals), index
    return type(structure)(vals), index


def pack_sequence_as(structure, flat_sequence):
    flat = list(flat_sequence)
    if len(flat) != len(flatten(structure)):
        raise ValueError("the flat sequence does not match the structure")
    return _pack(structure, flat, 0)[0]


def map_structure(func, *structure):
    flats = [flatten(s) for s in structure]
    return pack_sequence_as(structure[0], [func(*xs) for xs in zip(*flats)])


def assert_same_structure(nest1, nest2, check_types=True):
    if len(flatten(nest1)) != len(flatten(nest2)):
        raise ValueError("the two structures have different numbers of elements")


def convert_to_list(value, n, name, dtype=int):
    if isinstance(value, dtype):
        return [value] * n
    v = list(value)
    if len(v) != n:
        raise ValueError(f"The {name}'s length must be {n}, got {v}")
    return v
