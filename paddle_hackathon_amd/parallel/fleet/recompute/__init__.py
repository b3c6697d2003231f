"""``fleet.recompute`` (reference: python/paddle/distributed/fleet/recompute)."""
from ..utils import recompute, recompute_sequential  # noqa: F401

__all__ = ["recompute", "recompute_sequential"]
