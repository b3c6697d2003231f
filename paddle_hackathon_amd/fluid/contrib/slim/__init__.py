"""``fluid.contrib.slim`` (reference: python/paddle/fluid/contrib/slim): quantization."""
from . import quantization  # noqa: F401
