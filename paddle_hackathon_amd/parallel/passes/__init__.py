"""``paddle.distributed.passes`` (reference: python/paddle/distributed/passes/pass_base.py:21-320 —
PassContext, PassType, PassBase, register_pass, new_pass, PassManager; and the registered passes
of fuse_all_reduce.py, auto_parallel_{amp,fp16,recompute,gradient_merge,sharding}.py, cpp_pass.py).

A pass rewrites static Programs (main + startup lists) in place. The registered passes are
program rewrites over the per-op backward graph of static/backward.py:

* ``auto_parallel_amp``          loss scaling + check_finite_and_unscale + update_loss_scaling, the
                                 optimizer op skipped on overflow (static/passes.insert_loss_scaling)
* ``auto_parallel_fp16``         white-listed compute ops of the forward in fp16 / bf16
* ``auto_parallel_recompute``    recompute segments between ``checkpoints`` in the backward
* ``auto_parallel_gradient_merge_pass``  the optimizer op accumulates k_steps gradients and
                                 updates every k-th step (``avg``: the mean)
* ``auto_parallel_sharding``     optimizer state sharded over the data-parallel ranks: gradients
                                 reduced to each parameter's owner, owners update and broadcast
* ``fuse_all_reduce``            merges adjacent bucketed gradient all-reduces up to
                                 ``max_memory_size`` bytes (fewer, larger RCCL calls over xGMI)
* ``fuse_elewise_add_act`` / ``fuse_bn_act`` / ``fuse_bn_add_act`` / ``fuse_relu_depthwise_conv`` /
  ``fuse_optimizer`` / ``inplace_addto_op``: the reference turns on C++ graph fusions; on this
  backend those fusions are the kernels themselves (bias-GELU / BN-add-ReLU / multi-tensor
  optimizer HIP kernels), so the pass records the request on the program (``_build_flags``),
  which the executor's hipGraph path reads.
"""
from __future__ import annotations

import torch

from ...framework.core import Tensor, _wrap
from ...static import backward as B
from ...static import program as P

__all__ = ["new_pass", "PassManager", "PassContext", "PassBase", "PassType", "register_pass"]


class PassContext:
    def __init__(self):
        self._applied_passes = []
        self._attrs = {}

    def set_attr(self, key, value):
        self._attrs[key] = value

    def get_attr(self, key, default=None):
        return self._attrs.get(key, default)

    @property
    def passes(self):
        return self._applied_passes

    def _add_pass(self, pass_obj):
        self._applied_passes.append(pass_obj)

    def _pop_pass(self):
        del self._applied_passes[-1]


class PassType:
    UNKNOWN = 0
    COMM_OPT = 1
    CALC_OPT = 2
    PARALLEL_OPT = 3
    FUSION_OPT = 4


class PassBase:
    _REGISTERED_PASSES = {}
    _COMMON_RULES = []
    _BEFORE_WHITE_LISTS_DICT = {}
    _AFTER_WHITE_LISTS_DICT = {}
    name = None

    @staticmethod
    def _register(pass_name, pass_class):
        assert issubclass(pass_class, PassBase)
        PassBase._REGISTERED_PASSES[pass_name] = pass_class

    def __init__(self):
        self._attrs = {}

    def set_attr(self, key, value):
        self._attrs[key] = value
        return self

    def get_attr(self, key, default=None):
        return self._attrs.get(key, default)

    def _check_self(self):
        return True

    def _check_conflict(self, other_pass):
        return True

    def _type(self):
        return PassType.UNKNOWN

    def _check_conflict_including_common_rules(self, other_pass):
        return self._check_conflict(other_pass) and all(r(other_pass, self) for r in self._COMMON_RULES)

    def apply(self, main_programs, startup_programs, context=None):
        if context is None:
            context = PassContext()
        if not self._check_self():
            return context
        if not all(self._check_conflict_including_common_rules(p) for p in context.passes):
            return context
        mains = main_programs if isinstance(main_programs, (list, tuple)) else [main_programs]
        starts = startup_programs if isinstance(startup_programs, (list, tuple)) else [startup_programs]
        if len(starts) < len(mains):
            starts = list(starts) + [None] * (len(mains) - len(starts))
        self._apply_impl(mains, starts, context)
        context._add_pass(self)
        return context

    def _apply_impl(self, main_programs, startup_programs, context):
        for main, start in zip(main_programs, startup_programs):
            self._apply_single_impl(main, start, context)

    def _apply_single_impl(self, main_program, startup_program, context):
        raise NotImplementedError


def register_pass(name):
    def impl(cls):
        PassBase._register(name, cls)
        cls.name = name
        return cls
    return impl


def new_pass(name, pass_attrs={}):
    cls = PassBase._REGISTERED_PASSES.get(name)
    if cls is None:
        raise ValueError(f"Pass {name} is not registered (registered: {sorted(PassBase._REGISTERED_PASSES)})")
    p = cls()
    for k, v in (pass_attrs or {}).items():
        p.set_attr(k, v)
    return p


class PassManager:
    """applies a list of passes in order; with ``auto_solve_conflict`` a pass that conflicts with
    one applied earlier is skipped"""

    def __init__(self, passes, context=None, auto_solve_conflict=True):
        self._context = context if context is not None else PassContext()
        self._passes = list(passes)
        self._auto = auto_solve_conflict

    def apply(self, main_programs, startup_programs):
        ctx = self._context
        for p in self._passes:
            if self._auto and not all(p._check_conflict_including_common_rules(q) for q in ctx.passes):
                continue
            ctx = p.apply(main_programs, startup_programs, ctx)
        self._context = ctx
        return ctx

    @property
    def context(self):
        return self._context

    @property
    def names(self):
        return [p.name for p in self._passes]


# ------------------------------------------------------------------------------- helpers
def _optimize_ops(prog):
    return [op for op in prog.global_block().ops if B.op_role(op) == B.OPTIMIZE and "params" in op.kwargs]


def _params_grads(prog):
    out = []
    for op in _optimize_ops(prog):
        out += list(zip(op.kwargs["params"], op.kwargs["grads"]))
    return out


# ------------------------------------------------------------------------------- registered
@register_pass("auto_parallel_amp")
class AMPPass(PassBase):
    """attrs: loss (Variable), init_loss_scaling, incr_every_n_steps, decr_every_n_nan_or_inf,
    incr_ratio, decr_ratio, use_dynamic_loss_scaling — applied after backward + optimizer ops"""

    def _type(self):
        return PassType.CALC_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        from ...static import passes as SP
        loss = self.get_attr("loss")
        pg = _params_grads(main_program)
        if loss is None or not pg:
            raise ValueError("auto_parallel_amp needs attr 'loss' and a program with an optimizer op")
        opt_ops = _optimize_ops(main_program)
        blk = main_program.global_block()
        for op in opt_ops:   # the update moves behind the loss-scaling ops
            blk.ops.remove(op)
        new_pg, found, state = SP.insert_loss_scaling(
            main_program, loss, pg, init_scale=self.get_attr("init_loss_scaling", 32768.0),
            incr_every_n_steps=self.get_attr("incr_every_n_steps", 1000),
            decr_every_n_nan_or_inf=self.get_attr("decr_every_n_nan_or_inf", 2),
            incr_ratio=self.get_attr("incr_ratio", 2.0), decr_ratio=self.get_attr("decr_ratio", 0.8),
            dynamic=self.get_attr("use_dynamic_loss_scaling", True))
        unscaled = dict((id(p), g) for p, g in new_pg)
        for op in opt_ops:
            op.kwargs = dict(op.kwargs, grads=tuple(unscaled[id(p)] for p in op.kwargs["params"]), found_inf=found)
            blk.append_op(op)
        context.set_attr("found_inf", found)
        context.set_attr("loss_scaling", state)


@register_pass("auto_parallel_fp16")
class FP16Pass(PassBase):
    """attrs: dtype ('float16' | 'bfloat16'), custom_white_list"""

    def _type(self):
        return PassType.CALC_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        from ...static import passes as SP
        dt = torch.float16 if str(self.get_attr("dtype", "float16")) in ("float16", "fp16") else torch.bfloat16
        white = tuple(self.get_attr("custom_white_list", ()) or ()) + ("matmul", "linear", "conv2d", "bmm", "einsum",
                                                                        "mm")
        SP.cast_forward_to(main_program, dt, white)


@register_pass("auto_parallel_recompute")
class RecomputePass(PassBase):
    """attrs: checkpoints (Variables / names) — applied after append_backward"""

    def _type(self):
        return PassType.CALC_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        from ...static import passes as SP
        SP.recompute_segments(main_program, list(self.get_attr("checkpoints", []) or []))


def _merged_update(k_steps, avg, fn):
    state = {"n": 0, "acc": None}

    def update(params, grads, found_inf=None):
        if state["acc"] is None:
            state["acc"] = [torch.zeros_like(g._t, dtype=torch.float32) for g in grads]
        with torch.no_grad():
            for a, g in zip(state["acc"], grads):
                a.add_(g._t.float())
        state["n"] += 1
        if state["n"] % k_steps:
            return None
        merged = tuple(_wrap((a / k_steps if avg else a).to(g._t.dtype)) for a, g in zip(state["acc"], grads))
        for a in state["acc"]:
            a.zero_()
        return fn(params, merged, found_inf) if found_inf is not None else fn(params, merged)
    update.__name__ = getattr(fn, "__name__", "update")
    return update


@register_pass("auto_parallel_gradient_merge_pass")
class GradientMergePass(PassBase):
    """attrs: k_steps, avg"""

    def _type(self):
        return PassType.COMM_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        k = int(self.get_attr("k_steps", 1))
        avg = bool(self.get_attr("avg", True))
        if k <= 1:
            return
        for op in _optimize_ops(main_program):
            op.fn = _merged_update(k, avg, op.fn)
            op.attrs["gradient_merge_k_steps"] = k


@register_pass("auto_parallel_sharding")
class ShardingPass(PassBase):
    """attrs: sharding_degree (the data-parallel world), ring_id; the optimizer states of each
    parameter live on one owner rank (greedy size balance): gradients are reduced to the owner
    (c_reduce_coalesced), the owner updates, updated parameters are broadcast (c_broadcast)"""

    def _type(self):
        return PassType.COMM_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        import torch.distributed as tdist
        from ..fleet import static_optimizers as SO
        world = int(self.get_attr("sharding_degree", tdist.get_world_size() if tdist.is_initialized() else 1))
        rank = tdist.get_rank() if tdist.is_initialized() else 0
        ring = int(self.get_attr("ring_id", 0))
        if world <= 1:
            return
        blk = main_program.global_block()
        for op in _optimize_ops(main_program):
            params, grads = list(op.kwargs["params"]), list(op.kwargs["grads"])
            load = [0] * world
            owner = {}
            for i in sorted(range(len(params)), key=lambda i: -params[i]._t.numel()):
                r = min(range(world), key=lambda r: load[r])
                owner[i] = r
                load[r] += params[i]._t.numel()
            pos = blk.ops.index(op)
            new_g = list(grads)
            for r in range(world):
                idx = [i for i in range(len(params)) if owner[i] == r]
                if not idx:
                    continue
                outs = tuple(P._grad_var(blk, grads[i], grads[i].name + "@SHARD") for i in idx)
                red = P.OpDesc("c_reduce_coalesced", SO.c_reduce_coalesced, (),
                               {"xs": tuple(grads[i] for i in idx), "root": r, "ring_id": ring, "scale": 1.0 / world},
                               outs, attrs={"op_role": B.BACKWARD})
                for o in outs:
                    o.op = red
                blk.ops.insert(pos, red)
                pos += 1
                for i, o in zip(idx, outs):
                    new_g[i] = o
            mine = [i for i in range(len(params)) if owner[i] == rank]
            op.kwargs = dict(op.kwargs, params=tuple(params[i] for i in mine), grads=tuple(new_g[i] for i in mine))
            pos = blk.ops.index(op) + 1
            for r in range(world):
                idx = [i for i in range(len(params)) if owner[i] == r]
                if not idx:
                    continue
                bc = P.OpDesc("c_broadcast_coalesced", SO.c_broadcast_coalesced, (),
                              {"xs": tuple(params[i] for i in idx), "root": r, "ring_id": ring},
                              tuple(P.Variable(blk, params[i]._t.to("meta")) for i in idx),
                              attrs={"op_role": B.OPTIMIZE})
                blk.ops.insert(pos, bc)
                pos += 1
            opt = context.get_attr("optimizer")
            if opt is not None:
                opt._parameter_list = [params[i] for i in mine]


@register_pass("fuse_all_reduce")
class FuseAllReducePass(PassBase):
    """attrs: max_memory_size (bytes) — adjacent async gradient all-reduce buckets merged"""

    def _type(self):
        return PassType.COMM_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        from ..fleet import static_optimizers as SO
        limit = int(self.get_attr("max_memory_size", 128 * 2 ** 20))
        blk = main_program.global_block()
        starts = [op for op in blk.ops if op.type == "c_allreduce_start"]
        if len(starts) < 2:
            return
        waits = {op.kwargs["key"]: op for op in blk.ops if op.type == "c_allreduce_wait"}
        groups, cur, size = [], [], 0
        for st in starts:
            nb = sum(x._t.numel() * x._t.element_size() for x in st.kwargs["xs"])
            if cur and (size + nb > limit or st.kwargs["ring_id"] != cur[0].kwargs["ring_id"]
                        or st.kwargs["scale"] != cur[0].kwargs["scale"]):
                groups.append(cur)
                cur, size = [], 0
            cur.append(st)
            size += nb
        if cur:
            groups.append(cur)
        for g in groups:
            if len(g) == 1:
                continue
            last = g[-1]
            last.kwargs = dict(last.kwargs, xs=tuple(x for st in g for x in st.kwargs["xs"]))
            w_last = waits[last.kwargs["key"]]
            outs = []
            for st in g:
                w = waits[st.kwargs["key"]]
                outs += list(w.outputs)
                if st is not last:
                    blk.ops.remove(st)
                    blk.ops.remove(w)
            w_last.outputs = tuple(outs)
            for o in outs:
                o.op = w_last


class _BuildFlagPass(PassBase):
    """a reference C++ fusion pass: recorded on the program (its fusion is a HIP kernel here)"""

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        main_program.__dict__.setdefault("_build_flags", set()).add(self.name)


for _n in ("fuse_elewise_add_act", "fuse_bn_act", "fuse_bn_add_act", "fuse_relu_depthwise_conv", "fuse_optimizer",
           "inplace_addto_op"):
    register_pass(_n)(type(f"_{_n}", (_BuildFlagPass,), {}))
