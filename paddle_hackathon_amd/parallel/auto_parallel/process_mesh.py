"""ProcessMesh (reference: python/paddle/distributed/auto_parallel/process_mesh.py)."""
from __future__ import annotations

import numpy as np

__all__ = ["ProcessMesh", "get_default_mesh"]

_mesh_stack = []


def _device_type():
    import torch
    from ...framework import core
    dev = core.default_device()
    return "cuda" if getattr(dev, "type", "cpu") == "cuda" and torch.cuda.is_available() else "cpu"


class ProcessMesh:
    """An N-d array of process ids. ``ProcessMesh([[0, 1], [2, 3]], dim_names=["dp", "mp"])``.
    Used as a context manager it becomes the default mesh of ``shard_tensor`` / ``shard_op``."""

    def __init__(self, mesh, dim_names=None, parent=None):
        if isinstance(mesh, ProcessMesh):
            mesh = mesh.mesh.tolist()
        arr = np.asarray(mesh, dtype=np.int64)
        if arr.ndim == 0:
            raise ValueError("mesh must be a (nested) list of process ids")
        flat = arr.reshape(-1).tolist()
        if len(set(flat)) != len(flat) or min(flat) < 0:
            raise ValueError(f"process ids of a mesh must be unique and non-negative: {flat}")
        self._mesh = arr
        self._dim_names = list(dim_names) if dim_names is not None else [f"d{i}" for i in range(arr.ndim)]
        if len(self._dim_names) != arr.ndim:
            raise ValueError("one dim name per mesh dimension")
        self._device_mesh = None

    # reference-compatible accessors
    @property
    def mesh(self):
        return self._mesh

    @property
    def topology(self):
        return list(self._mesh.shape)

    shape = topology

    @property
    def processes(self):
        return self._mesh.reshape(-1).tolist()

    process_ids = processes

    @property
    def ndim(self):
        return self._mesh.ndim

    @property
    def dim_names(self):
        return list(self._dim_names)

    def dim_index(self, name):
        return self._dim_names.index(name) if isinstance(name, str) else int(name)

    def __contains__(self, rank):
        return int(rank) in self.processes

    def __eq__(self, other):
        return isinstance(other, ProcessMesh) and self.topology == other.topology and self.processes == other.processes

    def __ne__(self, other):
        return not self.__eq__(other)

    def __hash__(self):
        return hash((tuple(self.topology), tuple(self.processes)))

    def __str__(self):
        return f"ProcessMesh(shape={self.topology}, process_ids={self.processes}, dim_names={self._dim_names})"

    __repr__ = __str__

    def __enter__(self):
        _mesh_stack.append(self)
        return self

    def __exit__(self, *exc):
        _mesh_stack.pop()

    def device_mesh(self):
        """The torch DeviceMesh of this mesh (needs the process group of the job)."""
        if self._device_mesh is None:
            import torch
            from torch.distributed.device_mesh import DeviceMesh
            self._device_mesh = DeviceMesh(_device_type(), torch.as_tensor(self._mesh),
                                           mesh_dim_names=tuple(self._dim_names))
        return self._device_mesh


def get_default_mesh():
    if _mesh_stack:
        return _mesh_stack[-1]
    from .. import collective as C
    return ProcessMesh(list(range(max(1, C.get_world_size()))), dim_names=["dp"])
