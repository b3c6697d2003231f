"""``fluid.incubate`` (reference: python/paddle/fluid/incubate): ``fleet`` is the framework's
``paddle.distributed.fleet``."""
from ...parallel import fleet  # noqa: F401

__all__ = ["fleet"]
