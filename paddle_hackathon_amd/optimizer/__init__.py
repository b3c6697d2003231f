"""``paddle.optimizer`` (reference: python/paddle/optimizer/__init__.py)."""
from . import lr  # noqa: F401
from .optimizer import Optimizer, SGD, Momentum, Adam, AdamW, Adamax, Adagrad, Adadelta, RMSProp, Lamb  # noqa: F401

__all__ = ["Optimizer", "SGD", "Momentum", "Adam", "AdamW", "Adamax", "Adagrad", "Adadelta", "RMSProp", "Lamb"]
