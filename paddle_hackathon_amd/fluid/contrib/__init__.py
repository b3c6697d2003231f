"""``fluid.contrib`` (reference: python/paddle/fluid/contrib): the mixed-precision decorator
(``contrib.mixed_precision.decorate``), the 1.x ``BasicGRUUnit`` / ``BasicLSTMUnit`` and the
slim quantization passes (``contrib.slim``)."""
from . import mixed_precision  # noqa: F401
from .rnn_impl import BasicGRUUnit, BasicLSTMUnit  # noqa: F401
from . import slim  # noqa: F401
from . import layers  # noqa: F401
from .layers import *  # noqa: F401,F403
from . import extend_optimizer, model_stat, memory_usage_calc, op_frequence  # noqa: F401
from .extend_optimizer import extend_with_decoupled_weight_decay  # noqa: F401
from .memory_usage_calc import memory_usage  # noqa: F401
from .op_frequence import op_freq_statistic  # noqa: F401

__all__ = ["mixed_precision", "BasicGRUUnit", "BasicLSTMUnit", "extend_with_decoupled_weight_decay", "memory_usage",
           "op_freq_statistic"] + list(layers.__all__)
