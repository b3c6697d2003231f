"""``paddle.distributed.models`` (reference: python/paddle/distributed/models): ``moe``."""
from . import moe  # noqa: F401
