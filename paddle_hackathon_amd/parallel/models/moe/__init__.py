"""``paddle.distributed.models.moe`` (reference: python/paddle/distributed/models/moe/utils.py):
the expert-routing helpers of the framework's MoE (incubate.distributed.models.moe)."""
from ....incubate.distributed.models.moe import utils  # noqa: F401
from ....incubate.distributed.models.moe.utils import *  # noqa: F401,F403
