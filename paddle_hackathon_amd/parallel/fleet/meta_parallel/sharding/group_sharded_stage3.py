"""group_sharded_stage3 (reference module path)."""
from ....sharding import GroupShardedStage3  # noqa: F401

ShardingStage3 = GroupShardedStage3
