"""``fluid.contrib.layers`` (reference: python/paddle/fluid/contrib/layers/nn.py)."""
from .nn import *  # noqa: F401,F403
from .nn import __all__  # noqa: F401
