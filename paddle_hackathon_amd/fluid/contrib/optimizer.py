"""``fluid.contrib.optimizer`` (reference: python/paddle/fluid/contrib/optimizer.py): Momentum
with the regularization folded into the update (the framework's Momentum does that)."""
from ..optimizer import Momentum  # noqa: F401

__all__ = ["Momentum"]
