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

Static Programs take the reference's route: ``completion.py`` propagates the annotations through
the ops (per-op SPMD rules), ``planner.py`` picks replicate / column / row splits for the
weights nobody annotated by pricing candidate plans with the MI355X cost model,
``partitioner.py`` produces each rank's local Program with c_allgather / c_split / c_identity /
c_allreduce resharding ops, and ``parallelize`` ties them together (plus data-parallel gradient
sync and the optimizer step for training).
"""
from .process_mesh import ProcessMesh, get_default_mesh  # noqa: F401
from .interface import (shard_tensor, shard_op, dims_mapping_to_placements, placements_to_dims_mapping,  # noqa: F401
                        full_tensor, local_tensor)
from .reshard import Resharder, reshard  # noqa: F401
from .cost_model import estimate_cost  # noqa: F401
from .engine import Engine  # noqa: F401


def parallelize(program, fetches, process_mesh, rank=None, optimizer=None, loss=None, auto=False, mesh_dim=0,
                memory_limit=None, strategy=None):
    """Static-graph semi-/fully-automatic parallelism: (optionally plan) -> complete -> partition
    [-> per-op backward + the strategy's passes (recompute / amp / sharding / gradient merge) + gradient
    sync + optimizer]. Returns (local Program, local fetch Variables,
    Parallelizer). Feeds split along a mesh dim (annotated data) are fed as this rank's slice."""
    from .planner import plan
    from .partitioner import Parallelizer
    if auto:
        plan(program, process_mesh, mesh_dim, memory_limit)
    par = Parallelizer(program, process_mesh, rank)
    fetches = list(fetches)
    lidx = next((i for i, f in enumerate(fetches) if f is loss), len(fetches))
    prog, outs = par.parallelize(fetches + ([loss] if loss is not None and lidx == len(fetches) else []))
    if optimizer is not None:
        par.minimize(optimizer, outs[lidx], strategy)
    return prog, outs[:len(fetches)], par


def full_tensor_np(x):
    """numpy copy of the whole value of a (possibly distributed) tensor."""
    return full_tensor(x).detach().cpu().numpy()

__all__ = []
