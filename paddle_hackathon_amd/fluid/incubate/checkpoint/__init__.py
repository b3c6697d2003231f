"""``fluid.incubate.checkpoint`` (reference: python/paddle/fluid/incubate/checkpoint): the
auto-checkpoint implementation lives in ``paddle.incubate.checkpoint``."""
from . import auto_checkpoint  # noqa: F401
