"""sharding_stage2 (reference module path)."""
from ....sharding import GroupShardedStage2  # noqa: F401

ShardingStage2 = GroupShardedStage2
