"""``paddle.distributed.fleet.fleet_executor_utils`` (reference
python/paddle/distributed/fleet/fleet_executor_utils.py): TaskNode and the executor live in
``parallel/fleet_executor.py`` (native carrier)."""
from ..fleet_executor import FleetExecutor, TaskNode  # noqa: F401

__all__ = ["TaskNode", "FleetExecutor"]
