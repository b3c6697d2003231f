"""Resharding (reference: python/paddle/distributed/auto_parallel/reshard.py — the Resharder plans
send/recv, all-gather, split and concat ops between two distributed attributes of a tensor).

A layout is (process mesh, dims_mapping, partial mesh dims): tensor dim i is split along mesh dim
``dims_mapping[i]`` (-1: replicated), and a partial mesh dim means the ranks along it hold
addends of the value. ``plan`` turns a layout change into a list of per-mesh-dim steps, cheapest
first, and ``execute`` runs them on this rank's local block with differentiable collectives over
the 1-d process groups of the mesh (RCCL over xGMI on the GPU, gloo on CPU):

  partial on m, target splits dim j on m   -> reduce_scatter along j   (all_reduce + slice on gloo)
  partial on m otherwise                    -> all_reduce
  dim i split on m, target splits dim j     -> all_to_all (split j, concat i) when neither dim
                                               moves on another mesh dim, else gather + slice
  dim i split on m, target replicates on m  -> all_gather along i
  replicated on m, target splits dim j      -> local slice of j (no communication)

Gathers run before slices so nested splits never interleave. DTensors (dygraph auto-parallel
storage) are resharded through their local blocks with this plan and re-wrapped with the target
placements; static-partitioned local tensors (``dist_attr``) are resharded in place of their
block.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as tdist

from ...framework.core import Tensor, _wrap
from .interface import _as_mesh, _dims_mapping, dims_mapping_to_placements, shard_tensor

__all__ = ["Resharder", "reshard", "plan"]


class Step:
    __slots__ = ("kind", "mesh_dim", "src", "dst")

    def __init__(self, kind, mesh_dim, src=None, dst=None):
        self.kind, self.mesh_dim, self.src, self.dst = kind, mesh_dim, src, dst

    def __repr__(self):
        return f"{self.kind}(mesh_dim={self.mesh_dim}, src={self.src}, dst={self.dst})"


def _dim_on(dm, m):
    for i, v in enumerate(dm):
        if v == m:
            return i
    return None


def plan(src_dm, dst_dm, mesh_ndim, partial=()):
    """steps turning a block laid out as (src_dm, partial) into one laid out as dst_dm"""
    src_dm, dst_dm = list(src_dm), list(dst_dm)
    steps, cur = [], list(src_dm)
    for m in sorted(set(partial)):
        j = _dim_on(dst_dm, m)
        if j is not None and _dim_on(cur, m) is None and cur[j] == -1:
            steps.append(Step("reduce_scatter", m, dst=j))
            cur[j] = m
        else:
            steps.append(Step("all_reduce", m))
    gathers, swaps, slices = [], [], []
    for m in range(mesh_ndim):
        i, j = _dim_on(cur, m), _dim_on(dst_dm, m)
        if i == j:
            continue
        if i is not None and j is not None and cur[j] == -1 and dst_dm[i] == -1:
            swaps.append(Step("all_to_all", m, src=i, dst=j))
            continue
        if i is not None:
            gathers.append(Step("all_gather", m, src=i))
        if j is not None:
            slices.append(Step("slice", m, dst=j))
    return steps + gathers + swaps + slices


_GROUP_CACHE = {}


def _groups(mesh):
    """{mesh dim: (process group, ranks)} of the 1-d slices through this rank (created once per
    mesh, by every rank in the same order)"""
    key = (tuple(mesh.processes), tuple(mesh.topology))
    if key not in _GROUP_CACHE:
        arr = mesh.mesh
        rank = tdist.get_rank() if tdist.is_initialized() else 0
        out = {}
        for m in range(arr.ndim):
            for ranks in np.moveaxis(arr, m, -1).reshape(-1, arr.shape[m]).tolist():
                g = tdist.new_group(ranks) if tdist.is_initialized() and len(ranks) > 1 else None
                if rank in ranks:
                    out[m] = (g, ranks)
        _GROUP_CACHE[key] = out
    return _GROUP_CACHE[key]


def _gloo(group):
    return tdist.get_backend(group) == "gloo"


def _all_gather(t, dim, group, n):
    from torch.distributed.nn import functional as DF
    parts = DF.all_gather(t.contiguous(), group=group)
    return torch.cat(list(parts), dim=dim)


def _slice(t, dim, n, idx):
    size = t.shape[dim]
    assert size % n == 0, f"dim {dim} of size {size} does not split into {n}"
    return t.narrow(dim, idx * (size // n), size // n)


def execute(local, steps, mesh, rank=None):
    """run ``steps`` on this rank's block"""
    rank = rank if rank is not None else (tdist.get_rank() if tdist.is_initialized() else 0)
    coord = [int(c) for c in np.argwhere(mesh.mesh == rank)[0]]
    groups = _groups(mesh)
    from torch.distributed.nn import functional as DF
    t = local
    for s in steps:
        n = mesh.topology[s.mesh_dim]
        g = groups.get(s.mesh_dim, (None, [rank]))[0]
        me = coord[s.mesh_dim]
        if n == 1:
            continue
        if s.kind == "all_reduce":
            t = DF.all_reduce(t.contiguous(), group=g)
        elif s.kind == "reduce_scatter":
            if _gloo(g):
                t = _slice(DF.all_reduce(t.contiguous(), group=g), s.dst, n, me)
            else:
                ins = [c.contiguous() for c in t.chunk(n, dim=s.dst)]
                out = torch.empty_like(ins[0])
                t = DF.reduce_scatter(out, ins, group=g)
        elif s.kind == "all_gather":
            t = _all_gather(t, s.src, g, n)
        elif s.kind == "slice":
            t = _slice(t, s.dst, n, me).contiguous()
        elif s.kind == "all_to_all":
            if _gloo(g):     # gloo has no all_to_all: gather the blocks, keep this rank's pieces
                t = _slice(_all_gather(t, s.src, g, n), s.dst, n, me).contiguous()
            else:
                ins = [c.contiguous() for c in t.chunk(n, dim=s.dst)]
                outs = [torch.empty_like(ins[0]) for _ in range(n)]
                t = torch.cat(list(DF.all_to_all(outs, ins, group=g)), dim=s.src)
        else:
            raise ValueError(s.kind)
    return t


def _placements_to_layout(placements):
    from torch.distributed.tensor import Partial, Shard
    dm_of, partial = {}, []
    for m, p in enumerate(placements):
        if isinstance(p, Shard):
            dm_of[p.dim] = m
        elif isinstance(p, Partial):
            partial.append(m)
    return dm_of, partial


def reshard(x, process_mesh=None, shard_spec=None, dims_mapping=None):
    """Return ``x`` laid out as (process_mesh, shard_spec | dims_mapping); the input is unchanged."""
    mesh = _as_mesh(process_mesh)
    t = x._t if isinstance(x, Tensor) else x
    dm = _dims_mapping(t.dim(), mesh, dims_mapping, shard_spec)
    from torch.distributed.tensor import DTensor
    if isinstance(t, DTensor):
        dm_of, partial = _placements_to_layout(t.placements)
        src = [dm_of.get(i, -1) for i in range(t.dim())]
        local = execute(t.to_local(), plan(src, dm, mesh.ndim, partial), mesh)
        new = DTensor.from_local(local, mesh.device_mesh(), dims_mapping_to_placements(dm, mesh.ndim),
                                 run_check=False, shape=t.shape, stride=t.stride())
        out = _wrap(new)
        out.dist_attr = {"process_mesh": mesh, "dims_mapping": dm}
        return out
    attr = getattr(x, "dist_attr", None)
    if attr is not None and attr.get("local", False):
        # a static-partitioned local block: move it to the new layout
        src = list(attr["dims_mapping"])
        local = execute(t, plan(src, dm, mesh.ndim, attr.get("partial", ())), mesh)
        out = _wrap(local)
        out.dist_attr = {"process_mesh": mesh, "dims_mapping": dm, "local": True}
        return out
    return shard_tensor(_wrap(t), dist_attr={"dims_mapping": dm}, process_mesh=mesh)


class Resharder:
    """Reshard a set of tensors to target distributed attributes: ``Resharder(tensors, attrs).reshard()``
    (``attrs``: one ``{"process_mesh", "dims_mapping"}`` dict per tensor). ``plans()`` lists the
    steps each tensor needs (the reference Resharder's op insertion plan)."""

    def __init__(self, tensors=None, dist_attrs=None, rank_id=None, dist_context=None, *args, **kwargs):
        self.tensors = list(tensors or [])
        self.dist_attrs = list(dist_attrs or [])
        self.rank_id = rank_id

    def plans(self):
        out = []
        for t, a in zip(self.tensors, self.dist_attrs):
            mesh = _as_mesh(a.get("process_mesh"))
            src_attr = getattr(t, "dist_attr", None) or {}
            tt = t._t if isinstance(t, Tensor) else t
            src = list(src_attr.get("dims_mapping", [-1] * tt.dim()))
            dst = _dims_mapping(tt.dim(), mesh, a.get("dims_mapping"), None)
            out.append(plan(src, dst, mesh.ndim, src_attr.get("partial", ())))
        return out

    def reshard(self):
        return [reshard(t, a.get("process_mesh"), dims_mapping=a.get("dims_mapping"))
                for t, a in zip(self.tensors, self.dist_attrs)]
