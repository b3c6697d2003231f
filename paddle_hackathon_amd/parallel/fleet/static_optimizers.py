"""Static-graph (Program) distributed training: fleet meta-optimizers as program rewrites.

Reference: python/paddle/distributed/fleet/meta_optimizers/raw_program_optimizer.py:28 (gradient
all-reduce ops inserted between backward and optimizer ops, fused into buckets),
sharding_optimizer.py:46 (each rank owns a slice of the parameters: gradients are reduced to
the owner, only the owner updates, updated parameters are broadcast back),
gradient_merge_optimizer.py (gradients accumulate in persistable buffers; the optimizer ops
sit in a conditional block taken every k steps) and the c_allreduce_sum / c_reduce_sum /
c_broadcast collective ops (paddle/fluid/operators/collective/).

``minimize(loss)`` in static mode lays the step out as separate ops of the main Program:

    @backward(loss, params) -> grad Variables
    c_allreduce_coalesced(grads)              (DP: one RCCL call per bucket of <= bucket_mb)
  | c_reduce_coalesced(grads, owner)          (sharding: per owner, grads of its parameters)
    [gradient merge: accumulate; conditional_block every k steps around the update]
    @update(params, grads)                    (the inner optimizer on the given gradients)
    c_broadcast_coalesced(params, owner)      (sharding: owners send their updated slice)

so the communication is visible in the Program (``[op.type for op in prog.global_block().ops]``),
serialisable and editable like any other op. The collective op functions run
``torch.distributed`` (RCCL over xGMI on the GPU, gloo on CPU) on coalesced flat buffers.
"""
from __future__ import annotations

import torch
import torch.distributed as tdist

from ...framework import core as _core
from ...framework.core import Tensor, _wrap
from ...static import program as P
from ...static import control_flow as CF

_RINGS = {0: None}     # ring_id -> torch process group (0 = the global group)


def register_ring(ring_id, group):
    _RINGS[int(ring_id)] = group


def _group(ring_id):
    return _RINGS.get(int(ring_id))


def _flat(ts):
    return torch.cat([t.reshape(-1) for t in ts]) if len(ts) > 1 else ts[0].reshape(-1).clone()


def _unflat(buf, like):
    out, off = [], 0
    for t in like:
        n = t.numel()
        out.append(buf[off:off + n].view(t.shape))
        off += n
    return out


# ----------------------------------------------------------------------------- collective ops
def c_allreduce_coalesced(xs, ring_id=0, scale=1.0):
    """sum-all-reduce of a bucket of tensors in one call (flattened), then ``* scale``"""
    ts = [x._t for x in xs]
    buf = _flat([t.detach() for t in ts])
    if tdist.is_available() and tdist.is_initialized():
        tdist.all_reduce(buf, group=_group(ring_id))
    if scale != 1.0:
        buf.mul_(scale)
    return tuple(_wrap(t) for t in _unflat(buf, ts))


def c_reduce_coalesced(xs, root=0, ring_id=0, scale=1.0):
    """sum-reduce of a bucket to ``root`` (other ranks' results are unspecified, as in c_reduce_sum)"""
    ts = [x._t for x in xs]
    buf = _flat([t.detach() for t in ts])
    if tdist.is_available() and tdist.is_initialized():
        grp = _group(ring_id)
        dst = root if grp is None else tdist.get_global_rank(grp, root)
        tdist.reduce(buf, dst=dst, group=grp)
    if scale != 1.0:
        buf.mul_(scale)
    return tuple(_wrap(t) for t in _unflat(buf, ts))


def c_broadcast_coalesced(xs, root=0, ring_id=0):
    """broadcast a bucket of tensors from ``root`` and write them back in place (parameters)"""
    ts = [x._t for x in xs]
    if not (tdist.is_available() and tdist.is_initialized()):
        return tuple(xs)
    buf = _flat([t.detach() for t in ts])
    grp = _group(ring_id)
    src = root if grp is None else tdist.get_global_rank(grp, root)
    tdist.broadcast(buf, src=src, group=grp)
    with torch.no_grad():
        for t, v in zip(ts, _unflat(buf, ts)):
            t.copy_(v)
    return tuple(xs)


def gradient_merge_accumulate(grads, accs, step, k_steps=1, avg=True):
    """acc += g; returns (merged grads, take-update flag); the merged grads are acc (/k) on the
    k-th step (accumulators reset after use by ``gradient_merge_reset``)"""
    with torch.no_grad():
        for g, a in zip(grads, accs):
            a._t.add_(g._t.to(a._t.dtype))
        step._t.add_(1)
        take = bool(int(step._t.item()) % int(k_steps) == 0)
    merged = tuple(_wrap(a._t / k_steps if avg else a._t.clone()) for a in accs)
    return merged + (_wrap(torch.tensor(take)),)


def gradient_merge_reset(accs):
    with torch.no_grad():
        for a in accs:
            a._t.zero_()
    return _wrap(torch.zeros(()))


# ----------------------------------------------------------------------------- program building
def _op(blk, fn, kwargs, outs, type_=None):
    op = P.OpDesc(type_ or f"{fn.__module__}.{fn.__name__}", fn, (), kwargs, outs)
    for v in P._iter_vars(outs):
        v.op = op
    blk.append_op(op)
    return op


def _grad_vars(blk, params, suffix="@GRAD"):
    return tuple(P._grad_var(blk, p, p.name + suffix) for p in params)


def _buckets(items, bucket_bytes):
    out, cur, size = [], [], 0
    for it in items:
        nb = it._t.numel() * it._t.element_size()
        if cur and size + nb > bucket_bytes:
            out.append(cur)
            cur, size = [], 0
        cur.append(it)
        size += nb
    if cur:
        out.append(cur)
    return out


class StaticFleetOptimizer:
    """``fleet.distributed_optimizer(opt, strategy)`` in static mode."""

    def __init__(self, inner, strategy=None, world_size=None, rank=None):
        self.inner = inner
        self.strategy = strategy
        self.world = world_size if world_size is not None else (tdist.get_world_size() if tdist.is_initialized() else 1)
        self.rank = rank if rank is not None else (tdist.get_rank() if tdist.is_initialized() else 0)
        self.owner = {}

    def __getattr__(self, item):
        return getattr(self.inner, item)

    def _cfg(self, key, default):
        s = self.strategy
        if s is None:
            return default
        try:
            return getattr(s, key)
        except AttributeError:
            return default

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        prog = P.default_main_program()
        blk = prog.global_block()
        params = parameter_list if parameter_list is not None else [p for p in prog.all_parameters() if p.trainable]
        nog = {id(v) for v in (no_grad_set or []) if not isinstance(v, str)}
        params = [p for p in params if id(p) not in nog]
        sharding = bool(self._cfg("sharding", False)) and self.world > 1
        gm = bool(self._cfg("gradient_merge", False))
        fuse_mb = float((self._cfg("fuse_grad_size_in_MB", 32) or 32))
        # 1. backward: one op producing every gradient Variable
        gvars = _grad_vars(blk, params)

        def _backward(loss_t, *ps):
            gs = torch.autograd.grad(loss_t._t, [p._t for p in ps], allow_unused=True)
            return tuple(_wrap(g if g is not None else torch.zeros_like(p._t)) for g, p in zip(gs, ps))
        bwd = _op(blk, _backward, {}, gvars, "@backward")
        bwd.args = (loss,) + tuple(params)
        grads = list(gvars)
        # 2. gradient communication
        if self.world > 1 and not sharding:
            new = []
            for bucket in _buckets(grads, int(fuse_mb * 2 ** 20)):
                outs = _grad_vars(blk, [g for g in bucket], "@ALLREDUCE")
                _op(blk, c_allreduce_coalesced, {"xs": tuple(bucket), "ring_id": 0, "scale": 1.0 / self.world}, outs)
                new += list(outs)
            grads = new
        owned = list(range(len(params)))
        if sharding:
            # greedy size-balanced ownership (reference sharding/shard.py)
            load = [0] * self.world
            for i in sorted(range(len(params)), key=lambda i: -params[i]._t.numel()):
                r = min(range(self.world), key=lambda r: load[r])
                self.owner[i] = r
                load[r] += params[i]._t.numel()
            new = list(grads)
            for r in range(self.world):
                idx = [i for i in range(len(params)) if self.owner[i] == r]
                pos = {id(grads[i]): i for i in idx}
                for bucket in _buckets([grads[i] for i in idx], int(fuse_mb * 2 ** 20)):
                    outs = _grad_vars(blk, bucket, "@REDUCE")
                    _op(blk, c_reduce_coalesced, {"xs": tuple(bucket), "root": r, "ring_id": 0,
                                                  "scale": 1.0 / self.world}, outs)
                    for g, o in zip(bucket, outs):
                        new[pos[id(g)]] = o
            grads = new
            owned = [i for i in range(len(params)) if self.owner[i] == self.rank]
        # 3. the inner optimizer on the owned parameters
        opt = self.inner
        if opt._parameter_list is None:
            opt._add_param_group({"params": [params[i] for i in owned]})
            opt._parameter_list = [params[i] for i in owned]
        own_p = tuple(params[i] for i in owned)
        own_g = tuple(grads[i] for i in owned)

        def _update(*pg):
            n = len(pg) // 2
            ps, gs = pg[:n], pg[n:]
            for p, g in zip(ps, gs):
                p._t.grad = g._t.detach().to(p._t.dtype)
            with P._core_dynamic():
                opt.step()
            opt.clear_grad(set_to_zero=False)
            return None

        def append_update():
            u = _op(prog.current_block(), _update, {}, None, "@update")
            u.args = own_p + own_g

        if gm:
            k = int((self._cfg("gradient_merge_configs", {}) or {}).get("k_steps", 1))
            avg = bool((self._cfg("gradient_merge_configs", {}) or {}).get("avg", True))
            accs = tuple(_wrap(torch.zeros_like(p._t, dtype=torch.float32)) for p in own_p)
            step = _wrap(torch.zeros((), dtype=torch.int64))
            outs = tuple(P._grad_var(blk, p, p.name + "@MERGED") for p in own_p)
            flag = P.Variable(blk, torch.empty((), dtype=torch.bool, device="meta"))
            blk.vars[flag.name] = flag
            _op(blk, gradient_merge_accumulate, {"grads": own_g, "accs": accs, "step": step, "k_steps": k, "avg": avg},
                outs + (flag,))
            own_g = outs

            def true_fn():
                append_update()
                rv = P.Variable(prog.current_block(), torch.empty((), device="meta"))
                _op(prog.current_block(), gradient_merge_reset, {"accs": accs}, rv)
                return None
            CF.cond(flag, true_fn, lambda: None)
        else:
            append_update()
        # 4. sharding: owners broadcast their updated parameters
        if sharding:
            for r in range(self.world):
                idx = [i for i in range(len(params)) if self.owner[i] == r]
                for bucket in _buckets([params[i] for i in idx], int(fuse_mb * 2 ** 20)):
                    outs = tuple(P.Variable(blk, p._t.to("meta")) for p in bucket)
                    _op(blk, c_broadcast_coalesced, {"xs": tuple(bucket), "root": r, "ring_id": 0}, outs)
        return [op for op in blk.ops if op.type.startswith("@")], list(zip(params, gvars))

    def step(self):
        raise RuntimeError("static-mode distributed optimizer: use minimize(loss) and Executor.run")


def comm_op_types(program):
    return [op.type.rsplit(".", 1)[-1] for b in program.blocks for op in b.ops
            if op.type.rsplit(".", 1)[-1].startswith("c_")]
