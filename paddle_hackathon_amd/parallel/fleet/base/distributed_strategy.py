"""fleet.base.distributed_strategy (reference: .../fleet/base/distributed_strategy.py)."""
from ...strategy import DistributedStrategy  # noqa: F401
