"""``fluid.incubate`` (reference: python/paddle/fluid/incubate): ``fleet`` is the framework's
``paddle.distributed.fleet`` (also importable as the module ``fluid.incubate.fleet``), and
``checkpoint.auto_checkpoint`` the auto-checkpoint of ``paddle.incubate.checkpoint``."""
import sys as _sys

from ...parallel import fleet  # noqa: F401
from . import checkpoint  # noqa: F401

_sys.modules.setdefault(__name__ + ".fleet", fleet)

__all__ = ["fleet", "checkpoint"]
