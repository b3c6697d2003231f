"""``paddle.fluid.layers`` (reference: python/paddle/fluid/layers/__init__.py): the 1.x layer
functions, each with its 1.x signature and semantics, on the MI355X framework's tensors and
static Programs."""
from __future__ import annotations

from . import nn, tensor, control_flow, loss, detection, sequence_lod, learning_rate_scheduler, rnn, io, \
    metric_op, ops, distributions  # noqa: F401

_MODULES = (nn, tensor, control_flow, loss, detection, sequence_lod, learning_rate_scheduler, rnn, io, metric_op, ops,
            distributions)
from .nn import *  # noqa: F401,F403
from .tensor import *  # noqa: F401,F403
from .control_flow import *  # noqa: F401,F403
from .loss import *  # noqa: F401,F403
from .detection import *  # noqa: F401,F403
from .sequence_lod import *  # noqa: F401,F403
from .learning_rate_scheduler import *  # noqa: F401,F403
from .rnn import *  # noqa: F401,F403
from .io import *  # noqa: F401,F403
from .metric_op import *  # noqa: F401,F403
from .ops import *  # noqa: F401,F403
from .distributions import *  # noqa: F401,F403
from .control_flow import lod_rank_table  # noqa: F401
from ._common import act as _act  # noqa: F401

__all__ = []
for _m in _MODULES:
    __all__ += _m.__all__
