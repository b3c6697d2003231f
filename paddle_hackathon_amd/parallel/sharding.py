"""ZeRO-style sharding over flat bucketed storage (reference: python/paddle/distributed/sharding/
group_sharded.py; fleet/meta_parallel/sharding/{group_sharded_optimizer_stage2,group_sharded_stage2,
group_sharded_stage3,group_sharded_storage,group_sharded_utils}.py; fleet/meta_optimizers/
dygraph_optimizer/dygraph_sharding_optimizer.py).

Storage. Parameters are packed, per dtype and in backward (reverse registration) order, into flat
buckets of ``buffer_max_size`` elements (``group_sharded_storage.py:34-320`` ParamStorage /
GradStorage). Each bucket is padded to a multiple of ``nranks * 64`` elements and rank ``r`` owns
the contiguous slice ``[r * S, (r + 1) * S)`` of it — an element-wise ZeRO partition, so every rank
holds exactly 1/N of the optimizer state whatever the parameter sizes. The optimizer runs on
*pieces*: one view per (parameter, owning slice) that carries the parameter's name and attributes
(weight decay, lr ratio, need_clip), so per-parameter hyper-parameters and checkpoint keys keep
working; a rank's optimizer state for parameter ``p`` is its slice of ``p``.

Communication for xGMI (7 point-to-point links per MI355X, ring collectives per link): one
``reduce_scatter`` per gradient bucket, launched from the backward hook the moment the bucket's
last gradient is accumulated (overlapping the rest of backward), and one ``all_gather`` per
parameter bucket after the update — never a collective per parameter. Buckets default to 64 MB
of bf16 (2**25 elements), large enough that each ring step moves megabytes per link.

  * stage 1 (``os``):     optimizer state sharded. Gradients live in persistent flat bucket
                          buffers (``p.grad`` are views: zero-copy accumulation).
  * stage 2 (``os_g``):   + gradients sharded: each gradient is copied into a bucket buffer that
                          exists only until its reduce-scatter has completed; the full gradients
                          are freed as backward runs.
  * stage 3 (``p_g_os``): + parameters sharded. Each layer's parameters are one flat unit whose
                          1/N shard is all a rank keeps; the full unit is all-gathered just before
                          the layer's forward (and again before its backward), with the NEXT unit's
                          all-gather already in flight (prefetch, ``group_sharded_stage3.py:622``),
                          and freed after use. Parameters under ``segment_size`` elements stay
                          replicated (their gradients are all-reduced in one bucket).
                          ``offload=True`` keeps the fp32 master weights and moments of the shards
                          on the host (``group_sharded_stage3.py:71-151``).

The global-norm clip of the wrapped optimizer becomes sharding-aware (``group_sharded_utils.py:
47-119`` GroupShardedClipGrad): pieces are disjoint so their squared norms are summed over the
sharding group, replicated parameters are counted on one rank.
"""
from __future__ import annotations

import os

import contextlib
import math

import torch

from .recompute import queue_outer_callback as _queue_outer
import torch.distributed as dist

from ..framework.core import Tensor, Parameter, _wrap
from ..nn.layer.layers import Layer
from . import collective as C

__all__ = ["group_sharded_parallel", "save_group_sharded_model", "ShardingOptimizerStage1",
           "GroupShardedOptimizer", "GroupShardedStage2", "GroupShardedStage3", "comm_stats"]

_ALIGN = 64   # elements: every parameter / shard starts 128-B aligned (bf16) for the vector kernels

# per-process count of sharding collectives (tests assert the bucketed pattern)
comm_stats = {"reduce_scatter": 0, "all_gather": 0, "all_reduce": 0}


def _align(n, a=_ALIGN):
    return (n + a - 1) // a * a


def _bump_version(t):
    """Invalidate version-keyed derived copies (e.g. the cached transposed weights of
    ops/conv_gemm._wlayout) after a write that autograd cannot see (collective into the storage)."""
    try:
        torch.autograd.graph.increment_version(t)
    except Exception:   # pragma: no cover - older torch
        with torch.no_grad():
            t.add_(0)


def _pg(group):
    return group.pg if isinstance(group, C.Group) else group


class _Bucket:
    """A flat group of same-dtype parameters, padded to ``n * S`` elements; rank ``r`` owns
    ``[r * S, (r + 1) * S)``."""

    def __init__(self, params, n, rank, device, dtype):
        self.params = list(params)
        self.n, self.rank, self.device, self.dtype = n, rank, device, dtype
        self.offsets = []
        self.shapes = [tuple(p._t.shape) for p in self.params]
        self.numels = [p._t.numel() for p in self.params]
        off = 0
        for n_ in self.numels:
            self.offsets.append(off)
            off += _align(n_)
        self.off_of = {id(p): o for p, o in zip(self.params, self.offsets)}
        self.S = _align(-(-off // n))
        self.total = self.S * n
        self.lo, self.hi = rank * self.S, (rank + 1) * self.S
        self.flat_param = None     # full parameters (stage 1/2 persistent; stage 3 transient)
        self.flat_grad = None
        self.grad_shard = torch.zeros(self.S, dtype=dtype, device=device)
        self.ready = 0
        self.work = None
        self.pieces = []           # (param, piece Parameter, lo, hi) in flat coordinates

    def build_pieces(self, device=None, dtype=None, offload=False):
        """piece parameters over this rank's slice; their storage is the owning slice of
        ``flat_param`` (or a host fp32 copy when offloading)"""
        src = self.flat_param
        self.pieces = []
        for p, off, numel in zip(self.params, self.offsets, self.numels):
            lo, hi = max(off, self.lo), min(off + numel, self.hi)
            if lo >= hi:
                continue
            data = src[lo:hi]
            if offload:
                data = data.detach().to("cpu", torch.float32).clone().pin_memory() if torch.cuda.is_available() \
                    else data.detach().to("cpu", torch.float32).clone()
            piece = Parameter(data=data, name=p.name, trainable=not p.stop_gradient,
                              optimize_attr=getattr(p, "optimize_attr", {"learning_rate": 1.0}),
                              regularizer=getattr(p, "regularizer", None),
                              need_clip=getattr(p, "need_clip", True),
                              is_distributed=getattr(p, "is_distributed", False))
            piece._sharded_from = p
            self.pieces.append((p, piece, lo, hi))
        return [pc for _, pc, _, _ in self.pieces]

    def pack_params(self):
        """copy the current parameter values into a fresh flat buffer"""
        flat = torch.zeros(self.total, dtype=self.dtype, device=self.device)
        with torch.no_grad():
            for p, off in zip(self.params, self.offsets):
                flat[off:off + p._t.numel()].copy_(p._t.detach().reshape(-1))
        return flat

    def bind_params(self):
        for p, off, numel, shp in zip(self.params, self.offsets, self.numels, self.shapes):
            p._t.data = self.flat_param[off:off + numel].view(shp)

    def bind_grads(self):
        for p, off, numel, shp in zip(self.params, self.offsets, self.numels, self.shapes):
            if not p.stop_gradient:
                p._t.grad = self.flat_grad[off:off + numel].view(shp)


def _make_buckets(params, n, rank, max_elems):
    """group by dtype, in reverse registration order (≈ gradient-ready order), cut at max_elems"""
    by_dt = {}
    for p in reversed(list(params)):
        by_dt.setdefault(p._t.dtype, []).append(p)
    buckets = []
    for dt, ps in by_dt.items():
        cur, size = [], 0
        for p in ps:
            if cur and size + p._t.numel() > max_elems:
                buckets.append(_Bucket(cur, n, rank, cur[0]._t.device, dt))
                cur, size = [], 0
            cur.append(p)
            size += _align(p._t.numel())
        if cur:
            buckets.append(_Bucket(cur, n, rank, cur[0]._t.device, dt))
    return buckets


def _sharded_clip(optimizer, group, replicated=()):
    """make the optimizer's global-norm clip sum its squared norm over the sharding group
    (replicated parameters counted on the group's first rank only)"""
    from ..nn.clip import ClipGradByGlobalNorm
    clip = getattr(optimizer, "_grad_clip", None)
    if isinstance(clip, ClipGradByGlobalNorm) and group.nranks > 1:
        if clip._check_group is None:
            clip._check_group = _pg(group)
            clip._mp_degree = 1
    for p in replicated:   # counted once: first rank of the group (and of any tie it already has)
        p.is_firstly_shared = getattr(p, "is_firstly_shared", True) is not False and group.rank == 0


class GroupShardedOptimizer:
    """Stage 1 / 2 optimizer wrapper: owns the buckets, the backward hooks and the collectives.

    ``dp_group``: an extra data-parallel group (fleet dp x sharding): the reduce-scattered
    gradient shards are all-reduced over it. ``grads_sharded``: stage 2 (transient gradient
    buckets) instead of stage 1 (persistent flat gradient buffers)."""

    def __init__(self, optimizer, group, dp_group=None, grads_sharded=False, buffer_max_size=2 ** 25, offload=False,
                 hooks=True, replicate=()):
        self._inner = optimizer
        self._group = group
        self._pg = _pg(group)
        self._n = group.nranks
        self._rank = group.rank
        self._dp = dp_group if dp_group is not None and dp_group.nranks > 1 else None
        self._grads_sharded = grads_sharded
        self._offload = offload
        self._params = [p for p in optimizer._parameter_list]
        rep_ids = {id(p) for p in replicate}
        # replicated parameters (e.g. weights tied across pipeline stages): whole gradients,
        # all-reduced over the group, updated on every rank
        self._rep = [p for p in self._params if id(p) in rep_ids and not p.stop_gradient]
        self._train = [p for p in self._params if not p.stop_gradient and id(p) not in rep_ids]
        self._buckets = _make_buckets(self._train, self._n, self._rank, max(int(buffer_max_size), 1))
        self._pbucket = {}
        for b in self._buckets:
            b.flat_param = b.pack_params()
            b.bind_params()
            if not grads_sharded:
                b.flat_grad = torch.zeros(b.total, dtype=b.dtype, device=b.device)
                b.bind_grads()
            for p in b.params:
                self._pbucket[id(p._t)] = b
        pieces = []
        for b in self._buckets:
            pieces += b.build_pieces(offload=offload)
        # the inner optimizer now updates the pieces (its state is this rank's shard)
        optimizer._param_groups = [{"params": pieces + self._rep}]
        optimizer._parameter_list = pieces + self._rep
        _sharded_clip(optimizer, group, replicated=self._rep)
        self._sync = True
        self._queued = False
        self._handles = []
        if hooks:
            for p in self._train:
                self._handles.append(p._t.register_post_accumulate_grad_hook(self._make_hook(p)))

    # -- backward -------------------------------------------------------------------------------
    def _make_hook(self, p):
        key = id(p._t)

        def hook(t):
            b = self._pbucket[key]
            if self._grads_sharded:
                self._stash(b, p, t)
            if not self._sync:
                return
            if not self._queued:
                self._queued = True
                _queue_outer(self._finish)
            b.ready += 1
            if b.ready == len(b.params):
                self._launch(b)
        return hook

    def _stash(self, b, p, t):
        """stage 2: move the fresh gradient into the bucket buffer and free it"""
        if b.flat_grad is None:
            b.flat_grad = torch.zeros(b.total, dtype=b.dtype, device=b.device)
        off = b.off_of[id(p)]
        with torch.no_grad():
            b.flat_grad[off:off + t.numel()].add_(t.grad.reshape(-1))
        t.grad = None

    def _launch(self, b):
        scale = 1.0 / (self._n * (self._dp.nranks if self._dp is not None else 1))
        with torch.no_grad():
            b.flat_grad.mul_(scale)
        b.work = dist.reduce_scatter_tensor(b.grad_shard, b.flat_grad, group=self._pg, async_op=True)
        comm_stats["reduce_scatter"] += 1

    def _finish(self):
        self._queued = False
        for b in self._buckets:
            if b.work is None and b.ready == 0:
                continue
            if b.work is None:   # some parameters of the bucket got no gradient this step
                if b.flat_grad is None:
                    b.flat_grad = torch.zeros(b.total, dtype=b.dtype, device=b.device)
                self._launch(b)
        for b in self._buckets:
            if b.work is None:
                continue
            b.work.wait()
            b.work = None
            b.ready = 0
            if self._dp is not None:
                dist.all_reduce(b.grad_shard, group=_pg(self._dp))
                comm_stats["all_reduce"] += 1
            if self._grads_sharded:
                b.flat_grad = None   # the full gradient bucket is gone after the reduce-scatter
        self._allreduce_replicated()

    def _allreduce_replicated(self):
        grads = [p._t.grad for p in self._rep if p._t.grad is not None]
        if not grads:
            return
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat, group=self._pg)
        comm_stats["all_reduce"] += 1
        flat.mul_(1.0 / self._n)
        off = 0
        for g in grads:
            g.copy_(flat[off:off + g.numel()].view_as(g))
            off += g.numel()

    def _flush_grads(self):
        """reduce every bucket now (after gradients accumulated under ``no_sync``)"""
        for b in self._buckets:
            if b.work is None and (b.flat_grad is not None or not self._grads_sharded):
                self._launch(b)
                b.ready = len(b.params)
        self._finish()

    def no_sync(self):
        """accumulate gradients locally (gradient merge): no reduce-scatter until the context exits"""
        opt = self

        @contextlib.contextmanager
        def ctx():
            opt._sync = False
            try:
                yield
            finally:
                opt._sync = True
        return ctx()

    # -- step ---------------------------------------------------------------------------------
    def step(self):
        for b in self._buckets:
            for p, piece, lo, hi in b.pieces:
                g = b.grad_shard[lo - b.lo:hi - b.lo]
                piece._t.grad = g.to("cpu", torch.float32) if self._offload else g
        self._inner.step()
        with torch.no_grad():
            works = []
            for b in self._buckets:
                if self._offload:
                    for p, piece, lo, hi in b.pieces:
                        b.flat_param[lo:hi].copy_(piece._t.detach(), non_blocking=True)
                src = b.flat_param[b.lo:b.hi].clone()
                works.append(dist.all_gather_into_tensor(b.flat_param, src, group=self._pg, async_op=True))
                comm_stats["all_gather"] += 1
            for w in works:
                w.wait()
            for p in self._train:
                _bump_version(p._t)

    def minimize(self, loss=None, startup_program=None, parameters=None, no_grad_set=None):
        self.step()

    def clear_grad(self, set_to_zero=True):
        for b in self._buckets:
            b.grad_shard.zero_()
            if self._grads_sharded:
                b.flat_grad = None
            else:
                b.flat_grad.zero_()
                b.bind_grads()   # re-attach views a caller may have dropped
            for _, piece, _, _ in b.pieces:
                piece._t.grad = None
        for p in self._rep:
            if p._t.grad is not None:
                if set_to_zero:
                    p._t.grad.zero_()
                else:
                    p._t.grad = None

    clear_gradients = clear_grad

    def state_dict(self):
        return self._inner.state_dict()

    def set_state_dict(self, sd):
        return self._inner.set_state_dict(sd)

    def __getattr__(self, k):
        return getattr(self._inner, k)


def ShardingOptimizerStage1(optimizer, group, dp_group=None, reduce_grads=True, buffer_max_size=2 ** 25):
    """fleet's sharding stage 1 (DygraphShardingOptimizer): flat buckets, reduce-scatter +
    all-gather; ``reduce_grads=False`` builds the optimizer side of stage 2 (hooks installed by
    the caller)"""
    return GroupShardedOptimizer(optimizer, group, dp_group, grads_sharded=not reduce_grads,
                                 buffer_max_size=buffer_max_size)


class GroupShardedStage2(Layer):
    """Model wrapper for stage 2 (the optimizer wrapper does the work; kept for the reference API)."""

    def __init__(self, layer, sharding_optimizer, group=None, sync_buffers=False, buffer_max_size=2 ** 25):
        super().__init__()
        self._layer = layer
        self._opt = sharding_optimizer
        self._group = group

    def forward(self, *args, **kwargs):
        return self._layer(*args, **kwargs)

    def no_sync(self):
        return self._opt.no_sync()

    def state_dict(self, *a, **k):
        return self._layer.state_dict(*a, **k)

    def set_state_dict(self, *a, **k):
        return self._layer.set_state_dict(*a, **k)


class _Unit:
    """stage 3: the parameters owned directly by one sublayer, as one sharded flat buffer"""
    __slots__ = ("bucket", "layer", "full_work", "full_src", "ready", "grad_work", "grad_full", "gathered", "pieces")


class GroupShardedStage3(Layer):
    """Parameter + gradient + optimizer-state sharding with layer-ahead all-gather prefetch."""

    def __init__(self, layer, optimizer, group=None, sync_buffers=False, segment_size=2 ** 20, offload=False,
                 sync_comm=False, replicate=()):
        super().__init__()
        self._layer = layer
        self._group = group
        self._pg = _pg(group)
        self._n = group.nranks
        self._rank = group.rank
        self._offload = offload
        self._sync_comm = sync_comm
        self._optimizer = optimizer
        self._units = []
        self._punit = {}
        self._replicated = []
        seen = set()
        for sub in layer.sublayers(include_self=True):
            # a layer class with _sharding_unit = True (a transformer block whose forward reads its
            # sublayers' weights directly, fused kernels, never calling them) is ONE unit with all
            # of its parameters, gathered by its own hooks; otherwise each sublayer's own ones
            src = sub.parameters() if getattr(type(sub), "_sharding_unit", False) else sub._parameters.values()
            own = [p for p in src if p is not None and id(p) not in seen]
            for p in own:
                seen.add(id(p))
            rep_ids = {id(p) for p in replicate}
            big = [p for p in own if p._t.numel() >= segment_size and id(p) not in rep_ids]
            self._replicated += [p for p in own if p._t.numel() < segment_size or id(p) in rep_ids]
            by_dt = {}
            for p in big:
                by_dt.setdefault(p._t.dtype, []).append(p)
            for dt, ps in by_dt.items():
                u = _Unit()
                u.bucket = _Bucket(ps, self._n, self._rank, ps[0]._t.device, dt)
                u.layer = sub
                u.full_work = None
                u.full_src = None
                u.ready = 0
                u.grad_work = None
                u.grad_full = None
                u.gathered = False
                b = u.bucket
                full = b.pack_params()
                b.shard = full[b.lo:b.hi].clone()
                b.flat_param = full
                pieces = b.build_pieces(offload=offload)
                # the pieces must keep living in the persistent shard, not the transient full buffer
                for (p, piece, lo, hi) in b.pieces:
                    if not offload:
                        piece._t.data = b.shard[lo - b.lo:hi - b.lo]
                b.flat_param = None
                u.pieces = pieces
                self._units.append(u)
                for p in ps:
                    self._punit[id(p._t)] = u
                    p._t.data = torch.empty(0, dtype=p._t.dtype, device=p._t.device)
                    if not p.stop_gradient:
                        p._t.register_post_accumulate_grad_hook(self._make_grad_hook(u))
        self._uidx = {id(u): i for i, u in enumerate(self._units)}
        self._pool_off = {}
        self._init_pool()
        # replicated (small) parameters: one all-reduce bucket, updated on every rank
        self._rep_train = [p for p in self._replicated if not p.stop_gradient]
        self._rep_ready = 0
        for p in self._rep_train:
            p._t.register_post_accumulate_grad_hook(self._make_rep_hook())
        opt_params = [pc for u in self._units for pc in u.pieces] + self._replicated
        optimizer._param_groups = [{"params": opt_params}]
        optimizer._parameter_list = opt_params
        _sharded_clip(optimizer, group, replicated=self._replicated)
        self._order = []          # units in first-forward order (prefetch schedule)
        self._seen = set()
        self._order_pos = {}
        self._recording = True
        self._queued = False
        by_layer = {}
        for u in self._units:
            by_layer.setdefault(id(u.layer), []).append(u)
        for sub in layer.sublayers(include_self=True):
            us = by_layer.get(id(sub))
            if us:
                sub.register_forward_pre_hook(self._make_pre_fwd(us))
                sub.register_forward_post_hook(self._make_post_fwd(us))

    # -- gather buffers: one flat device pool carved by the native best-fit arena -------------
    def _init_pool(self):
        """Gathered units live in ONE pre-sized device buffer whose offsets come from the native
        coalescing allocator (csrc/runtime/arena.cpp): at 13B+ scale the gather/release churn of
        hundreds of MB-sized unit buffers per step then never fragments the caching allocator,
        and the peak is fixed up front. Capacity: the current unit + two prefetched ones of the
        largest size (layer-ahead prefetch, forward and backward), i.e. 3 x the largest unit.
        A request the pool cannot place falls back to a plain allocation (counted)."""
        self._arena = self._pool = None
        self._pool_fallbacks = 0
        # opt-in only: autograd keeps shallow copies / views of gathered weights in saved
        # activations, and an explicitly freed arena region is re-gathered into while they still
        # point at it (GPT blocks sharded at segment 64 trained differently from one process from
        # the second update on; plain allocations stay alive while referenced and match exactly —
        # tests/test_bench_layouts.py::test_stage3_sharded_blocks_with_recompute)
        if not self._units or os.environ.get("PHA_STAGE3_ARENA", "0") != "1":
            return
        try:
            from ..utils import native
            if not native.available():
                return
            dev = self._units[0].bucket.device
            largest = max(u.bucket.total * torch.empty(0, dtype=u.bucket.dtype).element_size() for u in self._units)
            cap = 3 * ((largest + 255) // 256 * 256)
            self._arena = native.Arena(cap, 256)
            self._pool = torch.empty(cap, dtype=torch.uint8, device=dev)
        except (OSError, RuntimeError, ValueError):
            self._arena = self._pool = None

    def _alloc_full(self, u):
        b = u.bucket
        nbytes = b.total * torch.empty(0, dtype=b.dtype).element_size()
        if self._arena is not None:
            try:
                off = self._arena.alloc(nbytes)
                self._pool_off[id(u)] = (off, nbytes)
                return self._pool[off:off + nbytes].view(b.dtype)
            except MemoryError:
                self._pool_fallbacks += 1
        return torch.empty(b.total, dtype=b.dtype, device=b.device)

    def _free_full(self, u):
        ent = self._pool_off.pop(id(u), None)
        if ent is not None:
            self._arena.free(ent[0])

    def pool_stats(self):
        if self._arena is None:
            return None
        return {"capacity": self._arena.capacity, "used": self._arena.used, "peak": self._arena.peak,
                "fallbacks": self._pool_fallbacks}

    # -- gather / release ---------------------------------------------------------------------
    def _issue_gather(self, u):
        if u.gathered or u.full_work is not None:
            return
        b = u.bucket
        b.flat_param = self._alloc_full(u)
        u.full_src = b.shard
        w = dist.all_gather_into_tensor(b.flat_param, b.shard, group=self._pg, async_op=not self._sync_comm)
        u.full_work = w if w is not None else True   # True: completed synchronously
        comm_stats["all_gather"] += 1

    def _gather(self, u):
        if u.gathered:
            return
        if u.full_work is None:
            self._issue_gather(u)
        if hasattr(u.full_work, "wait"):
            u.full_work.wait()
        u.full_work = None
        u.full_src = None
        u.bucket.bind_params()
        u.gathered = True

    def _release(self, u):
        if not u.gathered:
            if u.full_work is not None:   # a prefetch nobody consumed: drop it (its data may go stale)
                if hasattr(u.full_work, "wait"):
                    u.full_work.wait()
                u.full_work = None
                u.full_src = None
                u.bucket.flat_param = None
                self._free_full(u)
            return
        for p in u.bucket.params:
            p._t.data = torch.empty(0, dtype=p._t.dtype, device=p._t.device)
        u.bucket.flat_param = None
        self._free_full(u)
        u.gathered = False

    def _neighbor(self, u, step):
        if self._recording or not self._order:
            return None
        i = self._order_pos.get(id(u))
        if i is None:
            return None
        j = i + step
        return self._order[j] if 0 <= j < len(self._order) else None

    def _make_pre_fwd(self, units):
        def hook(layer, inputs):
            for u in units:
                if self._recording and id(u) not in self._seen:
                    self._seen.add(id(u))
                    self._order.append(u)
                self._gather(u)
            # layer-ahead prefetch — not when recompute re-runs the forward inside the backward:
            # the next layer's backward is already done, its gather would sit unconsumed
            if not self._recording and torch._C._current_graph_task_id() == -1:
                nxt = self._neighbor(units[-1], +1)
                if nxt is not None:
                    self._issue_gather(nxt)
        return hook

    def _make_post_fwd(self, units):
        def hook(layer, inputs, out):
            if torch.is_grad_enabled():
                # on EVERY output that needs a gradient: the backward may reach any of them first
                # (a block returning (h, m) runs m's nodes before h's hook fires); gathering is
                # idempotent
                outs = out if isinstance(out, (tuple, list)) else [out]
                for o in outs:
                    if isinstance(o, Tensor) and o._t.requires_grad:
                        o._t.register_hook(self._make_pre_bwd(units))
            for u in units:
                self._release(u)
            return None
        return hook

    def _make_pre_bwd(self, units):
        def hook(g):
            if not self._queued:
                self._queued = True
                _queue_outer(self._finish)
            for u in units:
                self._gather(u)
            prv = self._neighbor(units[0], -1)
            if prv is not None:
                self._issue_gather(prv)      # backward runs the layers in reverse
            return None
        return hook

    # -- gradients ----------------------------------------------------------------------------
    def _make_grad_hook(self, u):
        def hook(t):
            b = u.bucket
            if u.grad_full is None:
                u.grad_full = torch.zeros(b.total, dtype=b.dtype, device=b.device)
            off = b.off_of[id(self._param_of(u, t))]
            with torch.no_grad():
                u.grad_full[off:off + t.numel()].add_(t.grad.reshape(-1))
            t.grad = None
            u.ready += 1
            if u.ready == len([p for p in b.params if not p.stop_gradient]):
                u.ready = 0
                with torch.no_grad():
                    u.grad_full.mul_(1.0 / self._n)
                out = torch.empty(b.S, dtype=b.dtype, device=b.device)
                w = dist.reduce_scatter_tensor(out, u.grad_full, group=self._pg, async_op=True)
                comm_stats["reduce_scatter"] += 1
                u.grad_work = (w, out, u.grad_full)
                u.grad_full = None
                self._release(u)
        return hook

    def _param_of(self, u, t):
        for p in u.bucket.params:
            if p._t is t:
                return p
        raise KeyError("parameter not in unit")

    def _make_rep_hook(self):
        def hook(t):
            if not self._queued:
                self._queued = True
                _queue_outer(self._finish)
            self._rep_ready += 1
        return hook

    def _finish(self):
        self._queued = False
        if self._recording:
            self._recording = False
            self._order_pos = {id(u): i for i, u in enumerate(self._order)}
        for u in self._units:
            if u.grad_work is None:
                continue
            w, out, _keep = u.grad_work
            w.wait()
            u.grad_work = None
            for p, piece, lo, hi in u.bucket.pieces:
                g = out[lo - u.bucket.lo:hi - u.bucket.lo]
                if self._offload:
                    g = g.to("cpu", torch.float32)
                piece._t.grad = g.clone() if piece._t.grad is None else piece._t.grad.add_(g)
        # replicated parameters: one flat all-reduce (average)
        grads = [p._t.grad for p in self._rep_train if p._t.grad is not None]
        if grads and self._rep_ready:
            flat = torch.cat([g.reshape(-1) for g in grads])
            dist.all_reduce(flat, group=self._pg)
            comm_stats["all_reduce"] += 1
            flat.mul_(1.0 / self._n)
            off = 0
            for g in grads:
                g.copy_(flat[off:off + g.numel()].view_as(g))
                off += g.numel()
        self._rep_ready = 0

    # -- after the optimizer step -------------------------------------------------------------
    def _after_step(self):
        """offload: write the updated host fp32 pieces back into the device shards; bump the
        parameter versions so derived weight copies are recomputed next step"""
        with torch.no_grad():
            for u in self._units:
                self._release(u)   # a unit left gathered (no gradient this step) must re-gather fresh values
                if self._offload:
                    for p, piece, lo, hi in u.bucket.pieces:
                        u.bucket.shard[lo - u.bucket.lo:hi - u.bucket.lo].copy_(piece._t.detach(), non_blocking=True)
                for p in u.bucket.params:
                    _bump_version(p._t)

    def forward(self, *args, **kwargs):
        return self._layer(*args, **kwargs)

    def get_all_parameters(self):
        for u in self._units:
            self._gather(u)

    def state_dict(self, *a, **k):
        self.get_all_parameters()
        sd = self._layer.state_dict(*a, **k)
        out = {k2: _wrap(v._t.detach().clone()) for k2, v in sd.items()}
        for u in self._units:
            self._release(u)
        return out


class _Stage3Optimizer:
    """the optimizer returned for stage 3: runs the inner step on the shard pieces, then lets the
    model wrapper finish (offload copy-back, version bumps)"""

    def __init__(self, optimizer, model):
        self._inner = optimizer
        self._model = model

    def step(self):
        self._inner.step()
        self._model._after_step()

    def clear_grad(self, set_to_zero=True):
        self._inner.clear_grad(set_to_zero=False)
        for p in self._model._rep_train:
            p._t.grad = None

    clear_gradients = clear_grad

    def __getattr__(self, k):
        return getattr(self._inner, k)


def group_sharded_parallel(model, optimizer, level, scaler=None, group=None, offload=False, sync_buffers=False,
                           buffer_max_size=2 ** 25, segment_size=2 ** 20, sync_comm=False, replicate=()):
    """reference: python/paddle/distributed/sharding/group_sharded.py:group_sharded_parallel.
    ``buffer_max_size``: elements per flat bucket (stage 1/2); ``segment_size``: parameters with
    fewer elements stay replicated (stage 3); ``offload``: host fp32 optimizer state (stage 2/3);
    ``replicate``: parameters kept whole on every rank (weights tied across pipeline stages)."""
    if group is None:
        if not C.is_initialized():
            C.init_parallel_env()
        group = C.new_group(list(range(C.get_world_size())))
    from .data_parallel import sync_params_buffers
    sync_params_buffers(model, group, 0)
    if level == "os":
        if offload:
            raise ValueError("offload is supported with sharding levels 'os_g' and 'p_g_os' (as the reference)")
        opt = GroupShardedOptimizer(optimizer, group, grads_sharded=False, buffer_max_size=buffer_max_size,
                                    replicate=replicate)
        return model, opt, scaler
    if level == "os_g":
        opt = GroupShardedOptimizer(optimizer, group, grads_sharded=True, buffer_max_size=buffer_max_size,
                                    offload=offload, replicate=replicate)
        return GroupShardedStage2(model, opt, group, sync_buffers, buffer_max_size), opt, scaler
    if level == "p_g_os":
        m = GroupShardedStage3(model, optimizer, group, sync_buffers, segment_size, offload, sync_comm,
                               replicate=replicate)
        return m, _Stage3Optimizer(optimizer, m), scaler
    raise ValueError(f"unknown sharding level {level}")


def save_group_sharded_model(model, output, optimizer=None):
    import os
    from ..framework.io import save
    os.makedirs(output, exist_ok=True)
    sd = model.state_dict()
    if C.get_rank() == 0:
        save(sd, os.path.join(output, "model.pdmodel"))
    if optimizer is not None:
        save(optimizer.state_dict(), os.path.join(output, f"model.pdopt.rank{C.get_rank()}"))
