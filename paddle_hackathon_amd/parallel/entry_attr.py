"""``paddle.distributed.entry_attr`` (reference: python/paddle/distributed/entry_attr.py)."""
from . import ProbabilityEntry, CountFilterEntry, ShowClickEntry  # noqa: F401

__all__ = ["ProbabilityEntry", "CountFilterEntry", "ShowClickEntry"]
