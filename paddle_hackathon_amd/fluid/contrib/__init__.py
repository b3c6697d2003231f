"""``fluid.contrib`` (reference: python/paddle/fluid/contrib): the mixed-precision decorator
(``contrib.mixed_precision.decorate``) and ``BasicGRUUnit`` / ``BasicLSTMUnit``."""
from . import mixed_precision  # noqa: F401
from ..layers.rnn import GRUCell as BasicGRUUnit, LSTMCell as BasicLSTMUnit  # noqa: F401

__all__ = ["mixed_precision", "BasicGRUUnit", "BasicLSTMUnit"]
