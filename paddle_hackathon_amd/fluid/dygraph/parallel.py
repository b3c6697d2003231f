"""``fluid.dygraph.parallel`` (reference: python/paddle/fluid/dygraph/parallel.py)."""
from ...parallel.data_parallel import DataParallel  # noqa: F401
from ...parallel.collective import ParallelEnv, init_parallel_env

__all__ = ["prepare_context", "ParallelEnv", "DataParallel"]


def prepare_context(strategy=None):
    init_parallel_env()
    return strategy
