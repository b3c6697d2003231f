"""Semi-automatic parallelism (``paddle.distributed.auto_parallel``; reference:
python/paddle/distributed/auto_parallel/{interface,process_mesh,engine,reshard,cost_model}.py).

The reference annotates a static Program (``shard_tensor`` / ``shard_op``), completes the
distributed attributes of every op, partitions the program per rank and inserts reshard
communication. Here the same annotations drive PyTorch's distributed tensors: a
:class:`ProcessMesh` is a ``torch.distributed`` DeviceMesh over RCCL (gloo on CPU), an annotated
tensor becomes a DTensor whose placements come from ``dims_mapping`` (tensor dim i split along
mesh dim ``dims_mapping[i]``, -1 = replicated), op-level sharding propagation plays the role of
the completion pass and ``DTensor.redistribute`` the role of the resharder (all-gather /
reduce-scatter / all-to-all picked per placement change). :class:`Engine` runs the
prepare/fit/evaluate/predict loop on top.
"""
from .process_mesh import ProcessMesh, get_default_mesh  # noqa: F401
from .interface import (shard_tensor, shard_op, dims_mapping_to_placements, placements_to_dims_mapping,  # noqa: F401
                        full_tensor, local_tensor)
from .reshard import Resharder, reshard  # noqa: F401
from .cost_model import estimate_cost  # noqa: F401
from .engine import Engine  # noqa: F401


def full_tensor_np(x):
    """numpy copy of the whole value of a (possibly distributed) tensor."""
    return full_tensor(x).detach().cpu().numpy()

__all__ = []
