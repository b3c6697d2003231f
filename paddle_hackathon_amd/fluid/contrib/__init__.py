"""``fluid.contrib`` (reference: python/paddle/fluid/contrib): the mixed-precision decorator
(``contrib.mixed_precision.decorate``), the 1.x ``BasicGRUUnit`` / ``BasicLSTMUnit`` and the
slim quantization passes (``contrib.slim``)."""
from . import mixed_precision  # noqa: F401
from .rnn_impl import BasicGRUUnit, BasicLSTMUnit  # noqa: F401
from . import slim  # noqa: F401
from . import layers  # noqa: F401
from .layers import *  # noqa: F401,F403

__all__ = ["mixed_precision", "BasicGRUUnit", "BasicLSTMUnit"] + list(layers.__all__)
