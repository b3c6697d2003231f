"""``paddle.tensor.array`` (reference: python/paddle/tensor/array.py): tensor arrays."""
from ..fluid.layers.control_flow import create_array, array_write, array_read, array_length  # noqa: F401

__all__ = ["create_array", "array_write", "array_read", "array_length"]
