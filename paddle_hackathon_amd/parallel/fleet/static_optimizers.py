"""Static-graph (Program) distributed training: fleet meta-optimizers as program rewrites.

Reference: python/paddle/distributed/fleet/meta_optimizers/raw_program_optimizer.py:28 (gradient
all-reduce ops inserted between backward and optimizer ops, fused into buckets),
sharding_optimizer.py:46 (each rank owns a slice of the parameters: gradients are reduced to
the owner, only the owner updates, updated parameters are broadcast back),
gradient_merge_optimizer.py (gradients accumulate in persistable buffers; the optimizer ops
sit in a conditional block taken every k steps) and the c_allreduce_sum / c_reduce_sum /
c_broadcast collective ops (paddle/fluid/operators/collective/).

``minimize(loss)`` in static mode lays the step out as separate ops of the main Program:

    <op>_grad ... (one grad op per forward op, static/backward.py; recompute segments when
                   strategy.recompute gives checkpoints)
    c_allreduce_start(bucket)                 (DP: inserted right AFTER the last grad op of each
                                               bucket, async on the RCCL stream: the all-reduce of
                                               the late layers runs while the early layers' grad
                                               ops still compute — backward overlap)
  | c_reduce_coalesced(grads, owner)          (sharding: per owner, grads of its parameters)
    c_allreduce_wait(bucket)                  (before the update)
    [AMP: check_finite_and_unscale, update_loss_scaling; the update skipped on overflow]
    [gradient merge: accumulate; conditional_block every k steps around the update]
    <optimizer>(params, grads)                (the inner optimizer on the given gradients)
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


def c_allreduce_max(x, ring_id=0):
    """max-all-reduce of a scalar flag / tensor (the AMP found_infinite sync)"""
    t = x._t.detach()
    buf = t.reshape(-1).to(torch.float32).clone()
    if tdist.is_available() and tdist.is_initialized():
        tdist.all_reduce(buf, op=tdist.ReduceOp.MAX, group=_group(ring_id))
    out = buf.reshape(t.shape)
    return _wrap(out > 0 if t.dtype == torch.bool else out.to(t.dtype))


_ASYNC = {}   # id(start op) -> (work handle, flat buffer, tensors)


class _HostCounter:
    """a step counter the program carries by reference (the executor copies lists / dicts)"""
    __slots__ = ("n",)

    def __init__(self):
        self.n = 0


def c_allreduce_start(xs, ring_id=0, scale=1.0, key=0):
    """launch the sum-all-reduce of a bucket asynchronously (RCCL stream); c_allreduce_wait
    finishes it. Returns the bucket's tensors unchanged (the wait op produces the reduced ones)."""
    ts = [x._t.detach() for x in xs]
    buf = _flat(ts)
    work = None
    if tdist.is_available() and tdist.is_initialized():
        work = tdist.all_reduce(buf, group=_group(ring_id), async_op=True)
    _ASYNC[key] = (work, buf, ts, scale)
    return _wrap(torch.zeros(()))


def c_allreduce_wait(token, key=0):
    work, buf, ts, scale = _ASYNC.pop(key)
    if work is not None:
        work.wait()
    if scale != 1.0:
        buf.mul_(scale)
    return tuple(_wrap(t) for t in _unflat(buf, ts))


def gradient_merge_accumulate(grads, accs, step, k_steps=1, avg=True):
    """acc += g; returns (merged grads, take-update flag); the merged grads are acc (/k) on the
    k-th step (accumulators reset after use by ``gradient_merge_reset``). ``step`` is a host
    counter (the step count is known on the host: no device read, no sync)."""
    with torch.no_grad():
        for g, a in zip(grads, accs):
            a._t.add_(g._t.to(a._t.dtype))
    step.n += 1
    take = step.n % int(k_steps) == 0
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


def _buckets_idx(items, idx, bucket_bytes):
    """``_buckets`` over ``items`` returning the corresponding entries of ``idx``"""
    out, cur, size = [], [], 0
    for it, i in zip(items, idx):
        nb = it._t.numel() * it._t.element_size()
        if cur and size + nb > bucket_bytes:
            out.append(cur)
            cur, size = [], 0
        cur.append(i)
        size += nb
    if cur:
        out.append(cur)
    return out


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

    def __init__(self, inner, strategy=None, world_size=None, rank=None, comm=None):
        """comm = (ring id, group size, gradient scale): the data-parallel communication runs over that
        registered ring instead of the global group (auto_parallel's data mesh dim; world_size /
        rank are then the group's)"""
        self.inner = inner
        self.strategy = strategy
        self.world = world_size if world_size is not None else (tdist.get_world_size() if tdist.is_initialized() else 1)
        self.rank = rank if rank is not None else (tdist.get_rank() if tdist.is_initialized() else 0)
        self.comm = comm
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
        # 1. backward: per-op grad ops (+ recompute segments)
        from ...static import backward as B
        ckpts = None
        if bool(self._cfg("recompute", False)):
            ckpts = list((self._cfg("recompute_configs", {}) or {}).get("checkpoints", []) or [])
        pg = B.append_backward(loss, params, no_grad_set, checkpoints=ckpts or None)
        gvars = tuple(g for _, g in pg)
        grads = list(gvars)
        # AMP: loss scaling on the grad-op graph (check_finite_and_unscale + update_loss_scaling)
        self._found_inf = None
        if bool(self._cfg("amp", False)):
            from ...static import passes
            cfg = dict(self._cfg("amp_configs", {}) or {})
            pg2, self._found_inf, self._amp_state = passes.insert_loss_scaling(
                prog, loss, list(zip(params, grads)), init_scale=cfg.get("init_loss_scaling", 2.0 ** 15),
                incr_every_n_steps=cfg.get("incr_every_n_steps", 1000),
                decr_every_n_nan_or_inf=cfg.get("decr_every_n_nan_or_inf", 2),
                incr_ratio=cfg.get("incr_ratio", 2.0), decr_ratio=cfg.get("decr_ratio", 0.5),
                dynamic=cfg.get("use_dynamic_loss_scaling", True))
            grads = [g for _, g in pg2]
        # 2. gradient communication (tensor parallel: over the data-parallel group only, after the
        #    startup broadcasts that make replicated parameters equal — tensor_parallel_optimizer.py)
        ring, comm_world, scale = 0, self.world, 1.0 / max(1, self.world)
        tp = self._tensor_parallel(prog)
        if tp is not None:
            ring, comm_world = tp
            scale = 1.0 / comm_world
        if self.comm is not None:
            ring, comm_world, scale = self.comm
        if comm_world > 1 and not sharding:
            grads = self._insert_overlapped_allreduce(blk, grads, int(fuse_mb * 2 ** 20), ring, comm_world, scale)
        if self._found_inf is not None and (comm_world > 1 or sharding):
            self._sync_found_inf(blk, ring)
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
                    _op(blk, c_reduce_coalesced, {"xs": tuple(bucket), "root": r, "ring_id": ring,
                                                  "scale": scale}, outs)
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

        found_inf = self._found_inf

        def _update(*pg):
            n = len(pg) // 2
            ps, gs = pg[:n], pg[n:]
            if found_inf is not None and len(pg) % 2 == 1:   # AMP overflow: skip this update
                if bool(pg[-1]._t):
                    return None
                ps, gs = pg[:(len(pg) - 1) // 2], pg[(len(pg) - 1) // 2:-1]
            for p, g in zip(ps, gs):
                p._t.grad = g._t.detach().to(p._t.dtype)
            with P._core_dynamic():
                opt.step()
            opt.clear_grad(set_to_zero=False)
            return None

        def append_update():
            u = _op(prog.current_block(), _update, {}, None, type(opt).__name__.lower())
            u.args = own_p + own_g + ((found_inf,) if found_inf is not None else ())
            u.attrs["op_role"] = "optimize"

        if gm:
            k = int((self._cfg("gradient_merge_configs", {}) or {}).get("k_steps", 1))
            avg = bool((self._cfg("gradient_merge_configs", {}) or {}).get("avg", True))
            accs = tuple(_wrap(torch.zeros_like(p._t, dtype=torch.float32)) for p in own_p)
            step = _HostCounter()
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
                    _op(blk, c_broadcast_coalesced, {"xs": tuple(bucket), "root": r, "ring_id": ring}, outs)
        return [op for op in blk.ops if P.is_train_op(op)], list(zip(params, gvars))

    def _tensor_parallel(self, prog):
        """strategy.tensor_parallel: broadcast every replicated parameter (not ``is_distributed``) from
        the first rank of its model-parallel group and every parameter from the first rank of its
        data-parallel group (the reference's startup c_broadcast ops), register the data-parallel
        group as ring 2. -> (ring id, data-parallel degree) or None"""
        if not bool(self._cfg("tensor_parallel", False)) or not tdist.is_initialized():
            return None
        from .. import fleet as _fleet
        hcg = _fleet.fleet._hcg
        if hcg is None or hcg.get_model_parallel_world_size() <= 1:
            return None
        from .. import collective as C
        mp_g, dp_g = hcg.get_model_parallel_group(), hcg.get_data_parallel_group()
        with torch.no_grad():
            for p in prog.all_parameters():
                if not getattr(p, "is_distributed", False):
                    tdist.broadcast(p._t.data, src=mp_g.ranks[0], group=C._resolve_group(mp_g))
                if dp_g.nranks > 1:
                    tdist.broadcast(p._t.data, src=dp_g.ranks[0], group=C._resolve_group(dp_g))
        register_ring(2, C._resolve_group(dp_g))
        return 2, dp_g.nranks

    def _sync_found_inf(self, blk, ring):
        """every rank checked only its LOCAL gradients for inf/nan, before the all-reduce; an
        overflow on one rank reaches all of them through the sum. Max-all-reduce the flag over the
        gradient ring (the reference's c_allreduce_max on found_infinite,
        fleet/meta_optimizers/amp_optimizer.py + sharding's check group) and move
        update_loss_scaling behind it, so every rank skips the same step and keeps the same scale."""
        flag = self._found_inf
        synced = P.Variable(blk, torch.empty((), dtype=torch.bool, device="meta"), flag.name + "@GLOBAL")
        blk.vars[synced.name] = synced
        _op(blk, c_allreduce_max, {"x": flag, "ring_id": ring}, synced, "c_allreduce_max")
        upd = [op for op in blk.ops if op.type == "update_loss_scaling" and op.kwargs.get("found_inf") is flag]
        for op in upd:
            blk.ops.remove(op)
            op.kwargs = dict(op.kwargs, found_inf=synced)
            blk.append_op(op)
        self._found_inf = synced

    def _insert_overlapped_allreduce(self, blk, grads, bucket_bytes, ring=0, world=None, scale=None):
        """buckets in gradient-ready order (position of each grad's producing op); each bucket's
        async all-reduce starts right after its last grad op, and is waited for before the update"""
        pos = {id(op): i for i, op in enumerate(blk.ops)}
        ready = sorted(range(len(grads)), key=lambda i: pos.get(id(getattr(grads[i], "op", None)), len(blk.ops)))
        new = list(grads)
        inserts, waits = [], []
        for k, bucket_idx in enumerate(_buckets_idx([grads[i] for i in ready], ready, bucket_bytes)):
            bucket = tuple(grads[i] for i in bucket_idx)
            after = max(pos.get(id(getattr(g, "op", None)), len(blk.ops) - 1) for g in bucket)
            key = id(self) * 1000 + k
            tok = P.Variable(blk, torch.empty((), device="meta"))
            blk.vars[tok.name] = tok
            start = P.OpDesc("c_allreduce_start", c_allreduce_start, (),
                             {"xs": bucket, "ring_id": ring,
                              "scale": scale if scale is not None else 1.0 / (world or self.world), "key": key}, tok,
                             attrs={"op_role": "backward", "bucket": k})
            tok.op = start
            inserts.append((after, start))
            outs = _grad_vars(blk, list(bucket), "@ALLREDUCE")
            wait = P.OpDesc("c_allreduce_wait", c_allreduce_wait, (), {"token": tok, "key": key}, outs,
                            attrs={"op_role": "backward", "bucket": k})
            for o in outs:
                o.op = wait
            waits.append(wait)
            for i, o in zip(bucket_idx, outs):
                new[i] = o
        for after, op in sorted(inserts, key=lambda t: -t[0]):
            blk.ops.insert(after + 1, op)
        blk.ops.extend(waits)
        return new

    def step(self):
        raise RuntimeError("static-mode distributed optimizer: use minimize(loss) and Executor.run")


def comm_op_types(program):
    return [op.type.rsplit(".", 1)[-1] for b in program.blocks for op in b.ops
            if op.type.rsplit(".", 1)[-1].startswith("c_")]
