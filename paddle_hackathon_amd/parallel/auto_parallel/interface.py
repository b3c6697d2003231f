"""shard_tensor / shard_op (reference: python/paddle/distributed/auto_parallel/interface.py).

Both the 2.3 dict form (``dist_attr={"process_mesh": [[0, 1]], "dims_mapping": [0, -1]}``) and the
2.4 form (``process_mesh=mesh, shard_spec=["dp", None]``) are accepted. In static mode the
annotation is recorded on the Variable (``x.dist_attr``); in dygraph with a multi-process group
the tensor's storage becomes a DTensor laid out as annotated.
"""
from __future__ import annotations

from ...framework import core as _core
from ...framework.core import Tensor
from .process_mesh import ProcessMesh, get_default_mesh

__all__ = ["shard_tensor", "shard_op", "dims_mapping_to_placements", "placements_to_dims_mapping"]


def _as_mesh(m):
    if m is None:
        return get_default_mesh()
    return m if isinstance(m, ProcessMesh) else ProcessMesh(m)


def _dims_mapping(ndim, mesh, dims_mapping=None, shard_spec=None):
    if shard_spec is not None:
        if len(shard_spec) != ndim:
            raise ValueError(f"shard_spec {shard_spec} has {len(shard_spec)} entries for a {ndim}-d tensor")
        return [-1 if s is None else mesh.dim_index(s) for s in shard_spec]
    if dims_mapping is None:
        return [-1] * ndim
    dm = [int(d) for d in dims_mapping]
    if len(dm) != ndim or any(d < -1 or d >= mesh.ndim for d in dm):
        raise ValueError(f"dims_mapping {dm} invalid for a {ndim}-d tensor on a {mesh.ndim}-d mesh")
    used = [d for d in dm if d >= 0]
    if len(used) != len(set(used)):
        raise ValueError(f"a mesh dimension can shard only one tensor dimension: {dm}")
    return dm


def dims_mapping_to_placements(dims_mapping, mesh_ndim):
    """[tensor dim -> mesh dim] to DTensor placements [mesh dim -> Shard(tensor dim) | Replicate]."""
    from torch.distributed.tensor import Replicate, Shard
    pl = [Replicate() for _ in range(mesh_ndim)]
    for i, m in enumerate(dims_mapping):
        if m >= 0:
            pl[m] = Shard(i)
    return pl


def placements_to_dims_mapping(placements, ndim):
    from torch.distributed.tensor import Shard
    dm = [-1] * ndim
    for m, p in enumerate(placements):
        if isinstance(p, Shard):
            dm[p.dim] = m
    return dm


def _distributed():
    from .. import collective as C
    return C.is_initialized() and C.get_world_size() > 1


def _is_dtensor(t):
    from torch.distributed.tensor import DTensor
    return isinstance(t, DTensor)


def _apply(x, mesh, dm):
    """Lay ``x``'s storage out as (mesh, dims_mapping) (dygraph, multi-process)."""
    from torch.distributed.tensor import distribute_tensor
    dmesh = mesh.device_mesh()
    pl = dims_mapping_to_placements(dm, mesh.ndim)
    t = x._t
    is_param = isinstance(x, _core.Parameter)
    if _is_dtensor(t):
        new = t.redistribute(dmesh, pl)
        if is_param:
            new = new.detach().requires_grad_(not x.stop_gradient)
    else:
        new = distribute_tensor(t.detach() if is_param else t, dmesh, pl)
        if is_param:
            new = new.detach().requires_grad_(not x.stop_gradient)
    x._t = new
    return x


def shard_tensor(x, dist_attr=None, process_mesh=None, shard_spec=None):
    """Annotate (and in multi-process dygraph, lay out) ``x``: tensor dim ``i`` is split along
    mesh dim ``dims_mapping[i]`` (-1: replicated)."""
    if dist_attr is not None and not isinstance(dist_attr, dict):
        raise TypeError("dist_attr must be a dict with 'process_mesh' and/or 'dims_mapping'")
    dist_attr = dict(dist_attr or {})
    mesh = _as_mesh(process_mesh if process_mesh is not None else dist_attr.get("process_mesh"))
    ndim = len(x.shape)
    dm = _dims_mapping(ndim, mesh, dist_attr.get("dims_mapping"), shard_spec)
    try:
        x.dist_attr = {"process_mesh": mesh, "dims_mapping": dm}
    except AttributeError:
        pass
    if isinstance(x, Tensor) and _core.in_dynamic_mode() and _distributed():
        _apply(x, mesh, dm)
    return x


def shard_op(op_fn, dist_attr=None, process_mesh=None, in_shard_specs=None, out_shard_specs=None):
    """Wrap ``op_fn`` so its inputs are laid out as annotated before the call and its outputs
    after it. ``dist_attr`` (2.3 form) maps input/output tensors to ``{"dims_mapping": ...}`` and
    may carry a common ``process_mesh``; ``in_shard_specs`` / ``out_shard_specs`` (2.4 form) are
    lists of shard specs by position."""
    dist_attr = dict(dist_attr or {})
    mesh = _as_mesh(process_mesh if process_mesh is not None else dist_attr.get("process_mesh"))

    def spec_for(t, pos, specs):
        for k, v in dist_attr.items():
            if k is t and isinstance(v, dict):
                return v.get("dims_mapping"), None
        if specs is not None and pos < len(specs) and specs[pos] is not None:
            return None, specs[pos]
        return None, None

    def wrapped(*args, **kwargs):
        args = list(args)
        for i, a in enumerate(args):
            if isinstance(a, Tensor):
                dm, ss = spec_for(a, i, in_shard_specs)
                if dm is not None or ss is not None:
                    shard_tensor(a, process_mesh=mesh, shard_spec=ss,
                                 dist_attr=None if ss is not None else {"dims_mapping": dm})
        out = op_fn(*args, **kwargs)
        outs = out if isinstance(out, (list, tuple)) else [out]
        for i, o in enumerate(outs):
            if isinstance(o, Tensor) and out_shard_specs is not None and i < len(out_shard_specs) \
                    and out_shard_specs[i] is not None:
                shard_tensor(o, process_mesh=mesh, shard_spec=out_shard_specs[i])
        return out

    return wrapped


def full_tensor(x):
    """The whole (unsharded) value of a possibly-distributed tensor, as a plain torch tensor."""
    t = x._t if isinstance(x, Tensor) else x
    return t.full_tensor() if _is_dtensor(t) else t


def local_tensor(x):
    t = x._t if isinstance(x, Tensor) else x
    return t.to_local() if _is_dtensor(t) else t

