"""Distributed training (``paddle.distributed``): collectives on RCCL/xGMI, DataParallel,
fleet (hybrid DP/TP/PP/sharding), launch/spawn. ``paddle_hackathon_amd.distributed``
is an alias of this package."""
from .collective import *  # noqa: F401,F403
from .collective import _resolve_group  # noqa: F401
from .data_parallel import DataParallel, sync_params_buffers  # noqa: F401

try:  # optional subsystems (filled in progressively)
    from .spawn import spawn, launch  # noqa: F401
    from . import fleet  # noqa: F401
    from .mp_layers import split  # noqa: F401
    from .sharding import group_sharded_parallel, save_group_sharded_model  # noqa: F401
    from . import ps  # noqa: F401
    from . import auto_parallel  # noqa: F401
    from . import passes  # noqa: F401
    from .auto_parallel import shard_tensor, shard_op, ProcessMesh  # noqa: F401
except ImportError:  # pragma: no cover
    pass

ParallelMode = type("ParallelMode", (), {"DATA_PARALLEL": 0, "TENSOR_PARALLEL": 1, "PIPELINE_PARALLEL": 2, "SHARDING_PARALLEL": 3})


def gloo_init_parallel_env(rank_id, rank_num, server_endpoint):
    import os
    os.environ["RANK"], os.environ["WORLD_SIZE"] = str(rank_id), str(rank_num)
    host, port = server_endpoint.split(":")
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = host, port
    return init_parallel_env(backend="gloo")  # noqa: F405


def gloo_barrier():
    barrier()  # noqa: F405


def gloo_release():
    pass


class _Entry:
    def __init__(self, *args):
        self.args = args


class ProbabilityEntry(_Entry):
    pass


class CountFilterEntry(_Entry):
    pass


class ShowClickEntry(_Entry):
    pass


try:
    from .fleet.dataset import InMemoryDataset, QueueDataset  # noqa: E402,F401
except ImportError:  # pragma: no cover
    pass
