"""``fluid.trainer_factory`` (reference python/paddle/fluid/trainer_factory.py)."""
from ..static.trainer import TrainerFactory, FetchHandlerMonitor  # noqa: F401

__all__ = ["TrainerFactory", "FetchHandlerMonitor"]
