"""sharding_utils (reference module path): the group-sharded helpers."""
from ....sharding import group_sharded_parallel, save_group_sharded_model  # noqa: F401
