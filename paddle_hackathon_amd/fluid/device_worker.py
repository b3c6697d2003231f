"""``fluid.device_worker`` (reference python/paddle/fluid/device_worker.py): the dataset trainers'
per-thread workers, implemented in static/trainer.py."""
from ..static.trainer import DeviceWorker, Hogwild, DownpourSGD, DownpourSGDOPT, Section, HeterSection  # noqa: F401

__all__ = ["DeviceWorker", "Hogwild", "DownpourSGD", "DownpourSGDOPT", "Section", "HeterSection"]
