"""Partitioner + resharding: turn a completed (global) Program into this rank's local Program.

Reference: python/paddle/distributed/auto_parallel/partitioner.py:37 (Partitioner.partition: dist
ops produce the rank-local program, parameters sliced to local shards) and reshard.py (Resharder:
c_allgather / c_split / c_allreduce insertion where a tensor's mapping differs from what its
consumer needs), parallelizer_v2.py:38 (Parallelizer: completion -> partition -> reshard ->
backward / optimizer).

Per op of the serial Program, in order:
  * parameters / constants are sliced to the local block of their required mapping (cached);
  * Variable inputs whose current mapping differs from the required one are resharded
    (``c_allgather`` along a split dim that must become whole, ``c_split`` to take the local
    slice of a replicated value — free, no communication);
  * an input replicated along a mesh dim the op computes split over goes through ``c_identity``
    (identity forward, all-reduce of its gradient backward: the Megatron ``f`` operator);
  * the op runs on local shards (``reshape`` targets divided on split dims);
  * a partial-sum output is all-reduced over its mesh dims (``c_allreduce``; for a row-parallel
    linear the bias is added after the reduction).
Communication ops are autograd Functions over per-mesh-dim process groups (RCCL on the GPU, gloo
on CPU), so backward through the local Program is the distributed backward.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as tdist

from ...framework.core import Parameter, Tensor, _wrap
from ...static import program as P
from ...static.program import OpDesc, Program, Variable
from .completion import Completer, _resolve_shape, _short, dims_of

_GROUPS = {}     # mesh dim -> torch process group containing this rank (set by make_groups)
_NRANKS = {}


def make_groups(mesh, rank):
    """one process group per 1-d slice of ``mesh`` along each mesh dim (every rank creates all
    groups in the same order, as torch.distributed requires)"""
    arr = mesh.mesh
    for m in range(arr.ndim):
        moved = np.moveaxis(arr, m, -1).reshape(-1, arr.shape[m])
        for ranks in moved.tolist():
            g = tdist.new_group(ranks) if tdist.is_initialized() and len(ranks) > 1 else None
            if rank in ranks:
                _GROUPS[m] = g
                _NRANKS[m] = len(ranks)


def _coord(mesh, rank):
    idx = np.argwhere(mesh.mesh == rank)
    if not len(idx):
        raise ValueError(f"rank {rank} is not in {mesh}")
    return [int(c) for c in idx[0]]


# ----------------------------------------------------------------------------- comm functions
class _AllReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, mdim, avg):
        ctx.scale = 1.0 / _NRANKS.get(mdim, 1) if avg else 1.0
        out = t.clone()
        if _GROUPS.get(mdim) is not None:
            tdist.all_reduce(out, group=_GROUPS[mdim])
        return out * ctx.scale if avg else out

    @staticmethod
    def backward(ctx, g):
        return g * ctx.scale, None, None


class _Identity(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, mdim):
        ctx.mdim = mdim
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        g = g.clone()
        if _GROUPS.get(ctx.mdim) is not None:
            tdist.all_reduce(g, group=_GROUPS[ctx.mdim])
        return g, None


def _gather(t, dim, mdim):
    n = _NRANKS.get(mdim, 1)
    if n == 1 or _GROUPS.get(mdim) is None:
        return t
    parts = [torch.empty_like(t) for _ in range(n)]
    tdist.all_gather(parts, t.contiguous(), group=_GROUPS[mdim])
    return torch.cat(parts, dim)


def _local(t, dim, mdim, rank_in_group):
    n = _NRANKS.get(mdim, 1)
    if n == 1:
        return t
    return t.chunk(n, dim)[rank_in_group].contiguous()


class _Split(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, dim, mdim, idx):
        ctx.dim, ctx.mdim = dim, mdim
        return _local(t, dim, mdim, idx)

    @staticmethod
    def backward(ctx, g):
        return _gather(g, ctx.dim, ctx.mdim), None, None, None


class _AllGather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, dim, mdim, idx):
        ctx.dim, ctx.mdim, ctx.idx = dim, mdim, idx
        return _gather(t, dim, mdim)

    @staticmethod
    def backward(ctx, g):
        return _local(g, ctx.dim, ctx.mdim, ctx.idx), None, None, None


def c_allreduce(x, mesh_dim=0, avg=False):
    return _wrap(_AllReduce.apply(x._t, mesh_dim, avg))


def c_identity(x, mesh_dim=0):
    return _wrap(_Identity.apply(x._t, mesh_dim))


def c_split(x, dim=0, mesh_dim=0, index=0):
    return _wrap(_Split.apply(x._t, dim, mesh_dim, index))


def c_allgather(x, dim=0, mesh_dim=0, index=0):
    return _wrap(_AllGather.apply(x._t, dim, mesh_dim, index))


# ----------------------------------------------------------------------------- partitioner
def _q(fn):
    return f"{fn.__module__}.{fn.__name__}"


class Partitioner:
    def __init__(self, program, mesh, rank, completer=None):
        self.src = program
        self.mesh = mesh
        self.rank = rank
        self.coord = _coord(mesh, rank)
        self.comp = completer or Completer(mesh).complete(program)
        self.dst = Program()
        self.blk = self.dst.global_block()
        self.map = {}          # id(serial Variable) -> local Variable
        self.cur = {}          # id(local Variable) -> its dims_mapping
        self.params = {}       # (id(tensor), dm) -> local Parameter / constant
        self.comm = []         # inserted comm op types (introspection / tests)
        self.data_dims = set()

    # ------------------------------------------------------------------ helpers
    def _new_var(self, like_shape, dtype, name=None):
        v = Variable(self.blk, torch.empty(like_shape, dtype=dtype, device="meta"), name)
        self.blk.vars[v.name] = v
        return v

    def _emit(self, fn, kwargs, out_like, dm, type_=None):
        out = self._new_var(out_like._t.shape if isinstance(out_like, Tensor) else out_like,
                            out_like._t.dtype if isinstance(out_like, Tensor) else torch.float32)
        op = OpDesc(type_ or _q(fn), fn, (), kwargs, out)
        out.op = op
        self.blk.append_op(op)
        self.cur[id(out)] = list(dm)
        return out

    def local_shape(self, shape, dm):
        return [s // self.mesh.topology[m] if m >= 0 and s > 0 else s for s, m in zip(shape, dm)]

    def _slice_tensor(self, t, dm):
        key = (id(t), tuple(dm))
        if key in self.params:
            return self.params[key]
        data = t._t.detach()
        for i, m in enumerate(dm):
            if m >= 0:
                data = data.chunk(self.mesh.topology[m], i)[self.coord[m]]
        data = data.contiguous().clone()
        if isinstance(t, Parameter):
            loc = Parameter(data=data, name=t.name)
            loc.stop_gradient = t.stop_gradient
            loc.trainable = getattr(t, "trainable", True)
            loc.dist_attr = {"process_mesh": self.mesh, "dims_mapping": list(dm)}
            loc._serial = t
        else:
            loc = _wrap(data)
        self.params[key] = loc
        return loc

    def reshard(self, v, req):
        cur = list(self.cur[id(v)])
        for i, (c, r) in enumerate(zip(cur, req)):
            if c == r:
                continue
            if c >= 0:
                v = self._emit(c_allgather, {"x": v, "dim": i, "mesh_dim": c, "index": self.coord[c]}, v,
                               cur[:i] + [-1] + cur[i + 1:])
                self.comm.append("c_allgather")
                cur[i] = -1
            if r >= 0:
                v = self._emit(c_split, {"x": v, "dim": i, "mesh_dim": r, "index": self.coord[r]}, v,
                               cur[:i] + [r] + cur[i + 1:])
                self.comm.append("c_split")
                cur[i] = r
        return v

    # ------------------------------------------------------------------ main
    def partition(self, fetches):
        src_blk = self.src.global_block()
        for name, v in src_blk.vars.items():
            if getattr(v, "is_data", False):
                dm = self.comp.get(v)
                shp = v.declared_shape if v.declared_shape is not None else dims_of(v)
                loc = self._new_var([1 if s in (None, -1) else s for s in self.local_shape(
                    [(-1 if s is None else s) for s in shp], dm)], v._t.dtype, v.name)
                loc.is_data = True
                loc.declared_shape = self.local_shape([(-1 if s is None else s) for s in shp], dm)
                self.map[id(v)] = loc
                self.cur[id(loc)] = list(dm)
                self.data_dims |= {m for m in dm if m >= 0}
        for op in src_blk.ops:
            if P.is_train_op(op) or op.exec is not None:
                continue
            self._op(op)
        return self.dst, [self.map.get(id(f), f) for f in fetches]

    def _op(self, op):
        d = self.comp.ops[id(op)]
        name = _short(op.type)
        split_dims = {m for m in (d.output or []) if m >= 0} | set(d.partial)
        kw = {}
        for k, v in op.kwargs.items():
            req = d.inputs.get(k)
            if isinstance(v, Variable):
                lv = self.map[id(v)]
                if req is not None:
                    lv = self.reshard(lv, req)
                    for m in sorted(split_dims - {x for x in req if x >= 0}):
                        if self.mesh.topology[m] > 1 and lv._t.is_floating_point():
                            lv = self._emit(c_identity, {"x": lv, "mesh_dim": m}, lv, self.cur[id(lv)])
                            self.comm.append("c_identity")
                kw[k] = lv
            elif isinstance(v, Tensor) and req is not None:
                kw[k] = self._slice_tensor(v, req)
            elif isinstance(v, list) and any(isinstance(x, Variable) for x in v):
                kw[k] = [self.reshard(self.map[id(x)], [-1] * len(dims_of(x))) if isinstance(x, Variable) else x
                         for x in v]
            else:
                kw[k] = v
        if name == "reshape":
            osh = _resolve_shape(dims_of(op.kwargs["x"]), op.kwargs["shape"])
            tgt = list(op.kwargs["shape"])
            for j, m in enumerate(d.output):
                if m >= 0:
                    tgt[j] = osh[j] // self.mesh.topology[m] if tgt[j] not in (0,) else 0
            kw["shape"] = tgt
        bias = None
        if name == "linear" and d.partial and isinstance(kw.get("bias"), Tensor):
            bias = kw.pop("bias")
            kw["bias"] = None
        out = op.outputs
        if not isinstance(out, Variable):
            raise NotImplementedError(f"auto_parallel partitioner: multi-output op {op.type}")
        lv = self._emit(op.fn, kw, out, d.output if d.output is not None else [-1] * len(dims_of(out)), op.type)
        for m in d.partial:
            if self.mesh.topology[m] > 1:
                lv = self._emit(c_allreduce, {"x": lv, "mesh_dim": m, "avg": d.reduce == "avg"}, lv, self.cur[id(lv)])
                self.comm.append("c_allreduce")
        if bias is not None:
            from ...tensor import math as _m
            lv = self._emit(_m.add.__wrapped_op__ if hasattr(_m.add, "__wrapped_op__") else _m.add,
                            {"x": lv, "y": bias}, lv, self.cur[id(lv)], _q(_m.add))
        self.map[id(out)] = lv


class Parallelizer:
    """completion -> partition -> (backward + data-parallel gradient sync + optimizer) for one rank
    (reference parallelizer_v2.py)."""

    def __init__(self, program, mesh, rank=None, completer=None):
        self.rank = rank if rank is not None else (tdist.get_rank() if tdist.is_initialized() else 0)
        self.mesh = mesh
        make_groups(mesh, self.rank)
        self.part = Partitioner(program, mesh, self.rank, completer)

    def parallelize(self, fetches):
        prog, outs = self.part.partition(list(fetches))
        self.program = prog
        return prog, outs

    def local_parameters(self):
        return [p for p in self.part.params.values() if isinstance(p, Parameter) and not p.stop_gradient]

    def minimize(self, optimizer, loss, strategy=None):
        """training on the partitioned Program through the static fleet optimizer
        (parallel/fleet/static_optimizers.py): per-op grad ops on the local program, then the passes
        the reference runs on an auto-parallel program (distributed/passes/auto_parallel_*.py) —
        ``strategy.recompute`` (checkpoints), ``strategy.amp`` (loss scaling), gradient sync over the
        data-parallel mesh dim as bucketed all-reduces overlapped with the backward,
        ``strategy.sharding`` (optimizer-state owners along that dim) and
        ``strategy.gradient_merge`` — then the inner optimizer. The loss is already the global mean,
        so the data-parallel sync sums."""
        from ..fleet.static_optimizers import StaticFleetOptimizer, register_ring
        from ..strategy import DistributedStrategy
        params = self.local_parameters()
        dims = [m for m in sorted(self.part.data_dims) if self.mesh.topology[m] > 1]
        if len(dims) > 1 or any(m in p.dist_attr["dims_mapping"] for p in params for m in dims):
            return self._minimize_per_param(optimizer, loss)
        st = strategy if strategy is not None else DistributedStrategy()
        if dims:
            m = dims[0]
            ring = 100 + m
            register_ring(ring, _GROUPS.get(m))
            coord = _coord(self.mesh, self.rank)
            sfo = StaticFleetOptimizer(optimizer, st, world_size=self.mesh.topology[m], rank=coord[m],
                                       comm=(ring, self.mesh.topology[m], 1.0))
        else:
            sfo = StaticFleetOptimizer(optimizer, st, world_size=1, rank=0, comm=(0, 1, 1.0))
        with P.program_guard(self.program):
            sfo.minimize(loss, parameter_list=params)
        self.fleet_optimizer = sfo
        return params

    def _minimize_per_param(self, optimizer, loss):
        """several data-parallel mesh dims (or parameters split along one): @backward, one
        all-reduce per parameter over each data dim it is replicated on, @update"""
        from ..fleet.static_optimizers import _grad_vars, _op
        blk = self.program.global_block()
        params = self.local_parameters()
        gvars = _grad_vars(blk, params)

        def _backward(loss_t, *ps):
            gs = torch.autograd.grad(loss_t._t, [p._t for p in ps], allow_unused=True)
            return tuple(_wrap(g if g is not None else torch.zeros_like(p._t)) for g, p in zip(gs, ps))
        bwd = _op(blk, _backward, {}, gvars, "@backward")
        bwd.args = (loss,) + tuple(params)
        grads = list(gvars)
        for i, p in enumerate(params):
            dm = p.dist_attr["dims_mapping"]
            for m in sorted(self.part.data_dims - {x for x in dm if x >= 0}):
                if self.mesh.topology[m] > 1:
                    out = P._grad_var(blk, p, f"{p.name}@GRAD@DP{m}")
                    _op(blk, _grad_allreduce, {"x": grads[i], "mesh_dim": m}, out)
                    grads[i] = out
        if optimizer._parameter_list is None:
            optimizer._add_param_group({"params": params})
            optimizer._parameter_list = list(params)

        def _update(*pg):
            n = len(pg) // 2
            for p, g in zip(pg[:n], pg[n:]):
                p._t.grad = g._t.detach().to(p._t.dtype)
            with P._core_dynamic():
                optimizer.step()
            optimizer.clear_grad(set_to_zero=False)
        u = _op(blk, _update, {}, None, "@update")
        u.args = tuple(params) + tuple(grads)
        return params


def _grad_allreduce(x, mesh_dim=0):
    t = x._t.detach().clone()
    if _GROUPS.get(mesh_dim) is not None:
        tdist.all_reduce(t, group=_GROUPS[mesh_dim])
    return _wrap(t)


def gather_parameter(p, mesh):
    """the full (serial) value of a local parameter shard (all-gather along its split dims)"""
    t = p._t.detach()
    for i, m in enumerate(p.dist_attr["dims_mapping"]):
        if m >= 0:
            t = _gather(t, i, m)
    return t
