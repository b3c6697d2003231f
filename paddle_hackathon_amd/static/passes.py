"""Program passes over the per-op backward (static/backward.py).

``recompute_segments`` — static recompute (reference: python/paddle/fluid/backward.py
``_append_backward_ops_with_checkpoints_``, fleet/meta_optimizers/recompute_optimizer.py:20,
distributed/passes/auto_parallel_recompute.py): the forward ops between two checkpoints run without
keeping autograd state (``attrs["no_grad"]``); right before the grad ops of a segment, ``@RC``
copies of its forward ops are inserted that recompute the segment from its inputs, and the
segment's grad ops are rewired to differentiate the recomputed values. Checkpoint Variables (and
any other segment input produced inside another segment) enter a recomputation as fresh leaves
(``recompute_input``: detach + requires_grad), so every segment's backward stops at its own
inputs.

``amp_cast_grads`` / ``insert_loss_scaling`` — static AMP (reference
fleet/meta_optimizers/amp_optimizer.py:20, distributed/passes/auto_parallel_amp.py): the loss
gradient is seeded with the loss scale, every parameter gradient is unscaled and checked for
inf/nan in one fused op, and the optimizer op is skipped (``found_inf``) on overflow, with the
dynamic loss-scaling update of the reference's update_loss_scaling op.
"""
from __future__ import annotations

import torch

from ..framework.core import Tensor, _wrap
from . import program as P
from .backward import BACKWARD, FORWARD, LOSS, OPTIMIZE, _op_inputs, op_role


def _recompute_input(x):
    return _wrap(x._t.detach().requires_grad_(x._t.is_floating_point()))


def _grad_ops_of(prog):
    return prog.__dict__.setdefault("_grad_of", {})


def recompute_segments(prog, checkpoints):
    blk = prog.global_block()
    ck = [blk.vars.get(c, c) if isinstance(c, str) else c for c in checkpoints]
    ck_ids = {id(c) for c in ck}
    fwd = [op for op in blk.ops if op_role(op) == FORWARD]
    # segments: maximal runs of forward ops between checkpoint producers; a segment ends with the
    # op producing a checkpoint (its output is kept); the ops after the last checkpoint are not
    # recomputed (their backward follows immediately)
    segs, cur = [], []
    for op in fwd:
        cur.append(op)
        if any(id(o) in ck_ids for o in P._iter_vars(op.outputs)):
            segs.append(cur)
            cur = []
    if not segs:
        return prog
    grad_of = _grad_ops_of(prog)
    seg_of_op = {}
    for k, seg in enumerate(segs):
        for op in seg:
            seg_of_op[id(op)] = k
            op.attrs["no_grad"] = True
            op.attrs["recompute_segment"] = k
    produced_in_seg = {}
    for k, seg in enumerate(segs):
        for op in seg:
            for o in P._iter_vars(op.outputs):
                produced_in_seg[id(o)] = k
    ops = list(blk.ops)
    new_ops = []
    done = set()
    for op in ops:
        fop = grad_of.get(id(op))
        k = seg_of_op.get(id(fop)) if fop is not None else None
        if k is not None and k not in done:
            done.add(k)
            new_ops += _emit_recompute(prog, blk, segs[k], produced_in_seg, k)
        if k is not None:
            _rewire_grad_op(op, prog.__dict__["_rc_map"][k])
            clone = prog.__dict__["_rc_clone"][id(fop)]
            op.attrs["_fwd_id"] = id(clone)
            prog.__dict__.setdefault("_cut_ops", set()).add(id(clone))
        new_ops.append(op)
    blk.ops[:] = new_ops
    return prog


def _emit_recompute(prog, blk, seg, produced_in_seg, k):
    mp = {}
    out = []
    seg_ids = {id(o) for op in seg for o in P._iter_vars(op.outputs)}
    # inputs produced by a no-grad op (another segment's output, e.g. the previous checkpoint)
    for op in seg:
        for v in _op_inputs(prog, op):
            if isinstance(v, P.Variable) and id(v) not in seg_ids and id(v) in produced_in_seg and id(v) not in mp:
                leaf = P.Variable(blk, v._t, v.name + f"@RC{k}")
                blk.vars[leaf.name] = leaf
                rop = P.OpDesc("recompute_input", _recompute_input, (), {"x": v}, leaf,
                               attrs={"op_role": BACKWARD, "recompute_segment": k})
                leaf.op = rop
                out.append(rop)
                mp[id(v)] = leaf

    def remap(tree):
        if isinstance(tree, P.Variable):
            return mp.get(id(tree), tree)
        if isinstance(tree, list):
            return [remap(t) for t in tree]
        if isinstance(tree, tuple):
            return tuple(remap(t) for t in tree)
        if isinstance(tree, dict):
            return {kk: remap(v) for kk, v in tree.items()}
        return tree

    def fresh(tree):
        if isinstance(tree, P.Variable):
            nv = P.Variable(blk, tree._t, tree.name + f"@RC{k}")
            blk.vars[nv.name] = nv
            mp[id(tree)] = nv
            return nv
        if isinstance(tree, list):
            return [fresh(t) for t in tree]
        if isinstance(tree, tuple):
            return tuple(fresh(t) for t in tree)
        return tree

    for op in seg:
        if op.exec is not None:
            raise NotImplementedError("static recompute over control-flow ops")
        args, kwargs = remap(op.args), remap(op.kwargs)
        outs = fresh(op.outputs)
        attrs = {kk: v for kk, v in op.attrs.items() if kk != "no_grad"}
        attrs.update({"op_role": BACKWARD, "recompute_segment": k, "recompute_of": op.type})
        rop = P.OpDesc(op.type, op.fn, args, kwargs, outs, attrs=attrs)
        for o in P._iter_vars(outs):
            o.op = rop
        out.append(rop)
        prog.__dict__.setdefault("_rc_clone", {})[id(op)] = rop
    prog.__dict__.setdefault("_rc_map", {})[k] = mp
    return out


def _rewire_grad_op(gop, mp):
    kw = dict(gop.kwargs)
    kw["outs"] = tuple(mp.get(id(v), v) if isinstance(v, P.Variable) else v for v in kw["outs"])
    kw["ins"] = tuple(mp.get(id(v), v) if isinstance(v, P.Variable) else v for v in kw["ins"])
    gop.kwargs = kw


# ----------------------------------------------------------------------------- static AMP
def _scaled_ones(x, scale):
    return _wrap(torch.full_like(x._t, 1.0) * scale._t.to(x._t.dtype))


def _unscale_check(grads, scale):
    """grads / scale and one inf/nan flag over all of them (reference check_finite_and_unscale)"""
    inv = 1.0 / scale._t.float()
    outs, bad = [], torch.zeros((), dtype=torch.bool, device=scale._t.device)
    for g in grads:
        u = g._t.float() * inv
        bad = bad | ~torch.isfinite(u).all()
        outs.append(_wrap(u.to(g._t.dtype)))
    return tuple(outs) + (_wrap(bad),)


def _update_scaling(found_inf, scale, good, bad, incr_every, decr_every, incr_ratio, decr_ratio):
    """reference update_loss_scaling op, on device scalars (no host sync)"""
    with torch.no_grad():
        inf = found_inf._t.to(torch.int64)
        g = (good._t + 1) * (1 - inf)
        b = (bad._t + 1) * inf
        grow = (g >= incr_every).to(scale._t.dtype)
        shrink = (b >= decr_every).to(scale._t.dtype)
        s = scale._t * (1 + grow * (incr_ratio - 1)) * (1 + shrink * (decr_ratio - 1))
        scale._t.copy_(torch.clamp(s, min=1.0))
        good._t.copy_(g * (1 - grow.to(torch.int64)))
        bad._t.copy_(b * (1 - shrink.to(torch.int64)))
    return None


def insert_loss_scaling(prog, loss, params_grads, init_scale=2.0 ** 15, incr_every_n_steps=1000,
                        decr_every_n_nan_or_inf=2, incr_ratio=2.0, decr_ratio=0.5, dynamic=True):
    """rewrite: loss@GRAD seeded with the scale; grads unscaled + checked before the optimizer;
    returns (new params_grads, found_inf Variable, state dict)"""
    blk = prog.global_block()
    dev = loss._t.device if loss._t.device.type != "meta" else None
    from ..framework import core as _core
    dev = _core.default_device()
    scale = _wrap(torch.full((), float(init_scale), dtype=torch.float32, device=dev))
    good = _wrap(torch.zeros((), dtype=torch.int64, device=dev))
    bad = _wrap(torch.zeros((), dtype=torch.int64, device=dev))
    for op in blk.ops:
        if op_role(op) == LOSS and op.type == "fill_constant" and op.kwargs.get("x") is loss:
            op.fn = _scaled_ones
            op.kwargs = {"x": loss, "scale": scale}
            op.attrs["value"] = "loss_scaling"
            break
    else:
        raise RuntimeError("insert_loss_scaling: no loss@GRAD fill op (call append_backward first)")
    grads = tuple(g for _, g in params_grads)
    outs = tuple(P._grad_var(blk, g, g.name + "@UNSCALED") for g in grads)
    flag = P.Variable(blk, torch.empty((), dtype=torch.bool, device="meta"), "found_infinite")
    blk.vars[flag.name] = flag
    op = P.OpDesc("check_finite_and_unscale", _unscale_check, (), {"grads": grads, "scale": scale},
                  outs + (flag,), attrs={"op_role": BACKWARD})
    for o in outs + (flag,):
        o.op = op
    blk.append_op(op)
    if dynamic:
        blk.append_op(P.OpDesc("update_loss_scaling", _update_scaling, (),
                               {"found_inf": flag, "scale": scale, "good": good, "bad": bad,
                                "incr_every": incr_every_n_steps, "decr_every": decr_every_n_nan_or_inf,
                                "incr_ratio": incr_ratio, "decr_ratio": decr_ratio}, None,
                               attrs={"op_role": OPTIMIZE}))
    return [(p, o) for (p, _), o in zip(params_grads, outs)], flag, {"scale": scale, "good": good, "bad": bad}


def cast_forward_to(prog, dtype=torch.bfloat16, white=("matmul", "linear", "conv2d", "bmm", "einsum", "mm")):
    """O1-style static AMP: the white-listed compute ops of the forward run in ``dtype`` (inputs
    cast inside the op, output cast back to fp32), as the reference's fp16 rewrite inserts cast ops
    around white-list ops"""
    for op in prog.global_block().ops:
        if op_role(op) != FORWARD or op.exec is not None:
            continue
        name = op.type.rsplit(".", 1)[-1]
        if name in white and not op.attrs.get("amp_cast"):
            fn = op.fn

            def casted(*a, __fn=fn, **kw):
                def c(x):
                    if isinstance(x, Tensor) and x._t.is_floating_point():
                        return _wrap(x._t.to(dtype))
                    return x
                out = __fn(*[c(v) for v in a], **{k: c(v) for k, v in kw.items()})
                if isinstance(out, Tensor) and out._t.is_floating_point():
                    return _wrap(out._t.float())
                return out
            op.fn = casted
            op.attrs["amp_cast"] = str(dtype).replace("torch.", "")
    return prog
