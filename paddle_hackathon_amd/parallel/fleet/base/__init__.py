"""``paddle.distributed.fleet.base`` (reference: python/paddle/distributed/fleet/base): the role
makers, the strategy, the util and the Fleet class."""
from . import role_maker, distributed_strategy, util_factory, fleet_base, topology  # noqa: F401
