"""fleet.meta_parallel (reference: python/paddle/distributed/fleet/meta_parallel/__init__.py)."""
from ...mp_layers import (VocabParallelEmbedding, ColumnParallelLinear, RowParallelLinear, ParallelCrossEntropy,  # noqa: F401
                         RNGStatesTracker, get_rng_state_tracker, model_parallel_random_seed)
from ...pipeline import LayerDesc, SharedLayerDesc, PipelineLayer, PipelineParallel  # noqa: F401


def __getattr__(name):
    if name in ("TensorParallel", "ShardingParallel"):
        from .. import TensorParallel, ShardingParallel
        return {"TensorParallel": TensorParallel, "ShardingParallel": ShardingParallel}[name]
    raise AttributeError(name)
