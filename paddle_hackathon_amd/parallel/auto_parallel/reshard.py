"""Resharding (reference: python/paddle/distributed/auto_parallel/reshard.py — Resharder inserts
send/recv, all-gather, split and concat ops into a partitioned Program). Here a layout change is
``DTensor.redistribute``: Shard -> Replicate = all-gather, Partial -> Replicate = all-reduce,
Partial -> Shard = reduce-scatter, Shard(i) -> Shard(j) = all-to-all, over RCCL."""
from __future__ import annotations

from ...framework.core import Tensor, _wrap
from .interface import _as_mesh, _dims_mapping, dims_mapping_to_placements, shard_tensor

__all__ = ["Resharder", "reshard"]


def reshard(x, process_mesh=None, shard_spec=None, dims_mapping=None):
    """Return ``x`` laid out as (process_mesh, shard_spec | dims_mapping); the input is unchanged."""
    from torch.distributed.tensor import DTensor
    mesh = _as_mesh(process_mesh)
    t = x._t if isinstance(x, Tensor) else x
    dm = _dims_mapping(t.dim(), mesh, dims_mapping, shard_spec)
    if isinstance(t, DTensor):
        out = _wrap(t.redistribute(mesh.device_mesh(), dims_mapping_to_placements(dm, mesh.ndim)))
        out.dist_attr = {"process_mesh": mesh, "dims_mapping": dm}
        return out
    return shard_tensor(_wrap(t), dist_attr={"dims_mapping": dm}, process_mesh=mesh)


class Resharder:
    """Reshard a set of tensors to target distributed attributes: ``Resharder(tensors, attrs).reshard()``
    (``attrs``: one ``{"process_mesh", "dims_mapping"}`` dict per tensor)."""

    def __init__(self, tensors=None, dist_attrs=None, rank_id=None, dist_context=None, *args, **kwargs):
        self.tensors = list(tensors or [])
        self.dist_attrs = list(dist_attrs or [])
        self.rank_id = rank_id

    def reshard(self):
        return [reshard(t, a.get("process_mesh"), dims_mapping=a.get("dims_mapping"))
                for t, a in zip(self.tensors, self.dist_attrs)]
