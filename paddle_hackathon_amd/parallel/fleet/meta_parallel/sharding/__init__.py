"""``fleet.meta_parallel.sharding`` module paths (reference: python/paddle/distributed/fleet/
meta_parallel/sharding/): the group-sharded stages of parallel/sharding.py."""
from . import group_sharded_stage2, group_sharded_stage3, group_sharded_optimizer_stage2, group_sharded_utils  # noqa
from . import sharding_stage2, sharding_stage3, sharding_optimizer_stage2, sharding_utils  # noqa: F401
