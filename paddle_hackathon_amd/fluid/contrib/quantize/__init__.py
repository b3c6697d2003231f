"""``fluid.contrib.quantize`` (reference python/paddle/fluid/contrib/quantize)."""
from .quantize_transpiler import QuantizeTranspiler  # noqa: F401

__all__ = ["QuantizeTranspiler"]
