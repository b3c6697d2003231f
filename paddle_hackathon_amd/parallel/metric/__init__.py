"""``paddle.distributed.metric`` (reference: python/paddle/distributed/metric): metrics reduced
over the trainers (see ``fleet.metrics``)."""
from ..fleet.metrics import *  # noqa: F401,F403
