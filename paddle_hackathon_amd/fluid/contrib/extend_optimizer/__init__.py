"""``fluid.contrib.extend_optimizer`` (reference python/paddle/fluid/contrib/extend_optimizer)."""
from .extend_optimizer_with_weight_decay import extend_with_decoupled_weight_decay, DecoupledWeightDecay  # noqa: F401

__all__ = ["extend_with_decoupled_weight_decay"]
