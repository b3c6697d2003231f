"""``fluid.data`` (reference: python/paddle/fluid/data.py): a feed variable with exactly the
given shape (None / -1 for variable dims) — no implicit batch dimension, unlike layers.data."""
from .. import static as _static

__all__ = ["data"]


def data(name, shape, dtype="float32", lod_level=0):
    v = _static.data(name, [(-1 if s is None else s) for s in shape], dtype, lod_level)
    v.lod_level = lod_level
    return v
