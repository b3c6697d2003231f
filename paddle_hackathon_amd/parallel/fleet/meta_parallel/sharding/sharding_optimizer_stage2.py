"""sharding_optimizer_stage2 (reference module path)."""
from ....sharding import GroupShardedOptimizer  # noqa: F401

GroupShardedOptimizerStage2 = GroupShardedOptimizer
ShardingOptimizerStage2 = GroupShardedOptimizer
