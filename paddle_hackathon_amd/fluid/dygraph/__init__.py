"""``paddle.fluid.dygraph`` (reference: python/paddle/fluid/dygraph/__init__.py)."""
from . import base, layers, container, checkpoint, learning_rate_scheduler, jit, parallel, nn, rnn, io, amp  # noqa: F401
from .base import *  # noqa: F401,F403
from .layers import *  # noqa: F401,F403
from .container import *  # noqa: F401,F403
from .checkpoint import *  # noqa: F401,F403
from .learning_rate_scheduler import *  # noqa: F401,F403
from .jit import *  # noqa: F401,F403
from .parallel import *  # noqa: F401,F403
from .nn import *  # noqa: F401,F403
from .rnn import *  # noqa: F401,F403
from .io import *  # noqa: F401,F403
from .amp import *  # noqa: F401,F403
from ...framework.core import Tensor as VarBase  # noqa: F401

__all__ = []
for _m in (base, layers, container, checkpoint, learning_rate_scheduler, jit, parallel, nn, rnn, io, amp):
    __all__ += _m.__all__
