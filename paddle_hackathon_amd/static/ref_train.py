"""Writing a TRAINING Program as a reference ProgramDesc (reference: what append_backward and
Optimizer.minimize leave in ``main_program.desc`` — per-op ``<type>_grad`` ops with the forward's
input / output slots, ``<slot>@GRAD`` gradients, ``sum`` for gradient fan-in, ``fill_constant`` for
the loss gradient, and one optimizer op per parameter (sgd / momentum / adam / adamw) whose state
lives in persistable accumulators named ``{param}_{acc}_0``).

The grad ops carry no kernels of their own here: static/ref_grad.py reads ``<type>_grad`` back by
recomputing the forward op from its slots and taking the VJP, so a saved training program trains
after loading (tests/test_program_desc.py)."""
from __future__ import annotations

import torch

from ..framework.core import Tensor, _wrap
from . import proto as pb

__all__ = ["is_grad_op", "emit_grad", "emit_sum", "emit_fill_ones", "emit_assign", "emit_optimizer",
           "is_optimizer_op"]


def _bw():
    from . import backward
    return backward


def is_grad_op(program, op):
    return op.fn is _bw()._vjp and id(op) in program.__dict__.get("_grad_of", {})


def is_optimizer_op(op):
    return op.attrs.get("op_role") == "optimize" and "params" in op.kwargs and "optimizer" in op.attrs


def _tensors(v):
    if isinstance(v, Tensor):
        return [v]
    if isinstance(v, (list, tuple)):
        out = []
        for e in v:
            out += _tensors(e)
        return out
    return []


def fwd_slots(w, fop):
    """(type, {slot: [tensors]} inputs, {slot: [Variables]} outputs, {attr: value}) of the forward op as
    the writer emits it, or None when it has no reference form"""
    from .serialize import _REF, _fluid_ref, _qual_short, _EXTRA_ATTRS, _iter_vars, _derived_attrs
    from . import ref_emit
    short = _qual_short(fop.type)
    ref_op = fop.attrs.get("ref_op")
    if ref_op is not None:
        typ, r_ins, r_outs, r_attrs = ref_op
        return typ, {k: list(v) for k, v in r_ins.items()}, {k: list(v) for k, v in r_outs.items()}, dict(r_attrs)
    outs = list(_iter_vars(fop.outputs))
    spec = ref_emit.spec(short, fop)
    if spec is not None:
        typ, slot_of, out_slots, attrs, extra = spec
        ins = {}
        for k, v in fop.kwargs.items():
            if k in slot_of and _tensors(v):
                ins.setdefault(slot_of[k], []).extend(_tensors(v))
        for slot, t in extra.items():
            if t is not None and not slot.startswith("@out:"):
                ins.setdefault(slot, []).append(t)
        if isinstance(out_slots, tuple) and len(out_slots) == len(outs):
            o = {s: [v] for s, v in zip(out_slots, outs)}
        else:
            o = {out_slots if isinstance(out_slots, str) else out_slots[0]: outs}
        return typ, ins, o, dict(attrs)
    ref = _REF.get(short) or _fluid_ref(short)
    if ref is None or fop.args:
        return None
    typ, slot_of, out_slot, attr_map = ref
    ins, attrs = {}, {}
    for k, v in fop.kwargs.items():
        ts = _tensors(v)
        if ts:
            ins.setdefault(slot_of.get(k, k), []).extend(ts)
        elif v is not None:
            attrs[attr_map.get(k, k)] = v
    attrs.update(_EXTRA_ATTRS.get(short, {}))
    attrs.update(_derived_attrs(short, fop.kwargs))
    return typ, ins, {out_slot: outs}, attrs


def emit_grad(w, program, op, msg, ins, outs):
    """the reference <type>_grad op of a recorded grad op (static/backward.py _vjp)"""
    from .serialize import _set_attr
    fop = program.__dict__["_grad_of"][id(op)]
    spec = fwd_slots(w, fop)
    if spec is None:
        raise NotImplementedError(f"training program: {fop.type} has no reference op type, so its grad op "
                                  "cannot be written")
    typ, f_ins, f_outs, attrs = spec
    msg.type = typ + "_grad"
    slot_of_in = {}
    for slot, ts in f_ins.items():
        ins[slot] = [w.tensor_name(t) for t in ts]
        for t in ts:
            slot_of_in.setdefault(id(t), slot)
    out_slot_of = {}
    for slot, vs in f_outs.items():
        ins[slot] = [w.tensor_name(v) for v in vs]   # Out etc.: the output-based grad makers read it
        for v in vs:
            out_slot_of[id(v)] = slot
    for o, g in zip(op.kwargs["outs"], op.kwargs["gouts"]):
        if g is None or id(o) not in out_slot_of:
            continue
        ins.setdefault(out_slot_of[id(o)] + "@GRAD", []).append(w.tensor_name(g))
    # one gradient per input position ("@EMPTY@" where none is wanted); an input used at several
    # positions (x * x) gets one partial per position, summed by a following `sum` op (the
    # reference backward's @RENAME@ + sum)
    want = {id(v): g for v, g in zip(op.kwargs["ins"], op.outputs)}
    for v in op.kwargs["ins"]:
        if id(v) not in slot_of_in:
            raise NotImplementedError(f"training program: {fop.type}_grad: input {getattr(v, 'name', v)} has no slot")
    uses = {}
    for ts in f_ins.values():
        for t in ts:
            uses[id(t)] = uses.get(id(t), 0) + 1
    partials = {}
    for slot, ts in f_ins.items():
        names = []
        for t in ts:
            g = want.get(id(t))
            if g is None:
                names.append("@EMPTY@")
            elif uses[id(t)] > 1:
                from . import ref_emit
                lst = partials.setdefault(id(t), (g, []))[1]
                tmp = ref_emit._tmp_var(f"{w.tensor_name(g)}@RENAME@{len(lst)}", g, list(g.declared_shape or g.shape)
                                        if hasattr(g, "declared_shape") else list(g.shape))
                lst.append(tmp)
                names.append(w.tensor_name(tmp))
            else:
                names.append(w.tensor_name(g))
        if any(n != "@EMPTY@" for n in names):
            outs[slot + "@GRAD"] = names
    for k, v in attrs.items():
        _set_attr(msg, k, v)
    _set_attr(msg, "op_role", 1)
    w._pending_parts = [("sum", {"X": lst}, {"Out": [g]}, {}) for g, lst in partials.values()]


def emit_sum(w, op, msg, ins, outs):
    from .serialize import _set_attr
    msg.type = "sum"
    ins["X"] = [w.tensor_name(t) for t in op.kwargs["xs"]]
    outs["Out"] = [w.tensor_name(op.outputs)]
    _set_attr(msg, "op_role", 1)


def emit_assign(w, op, msg, ins, outs):
    from .serialize import _set_attr
    msg.type = "assign"
    ins["X"] = [w.tensor_name(op.kwargs["x"])]
    outs["Out"] = [w.tensor_name(op.outputs)]
    _set_attr(msg, "op_role", 1)


def emit_fill_ones(w, op, msg, ins, outs):
    """the loss gradient: fill_constant of the loss's shape (the reference's op_role 257)"""
    from .serialize import _set_attr
    x = op.kwargs["x"]
    msg.type = "fill_constant"
    outs["Out"] = [w.tensor_name(op.outputs)]
    shape = [int(s) for s in (x._t.shape or [1])]
    _set_attr(msg, "shape", shape)
    _set_attr(msg, "value", 1.0)
    _set_attr(msg, "dtype", pb.vartype_of(x._t.dtype))
    _set_attr(msg, "op_role", 257)


def _named(t, name):
    t.name = name
    t._pha_persist_name = True
    return t


def emit_optimizer(w, op, block_msg):
    """one reference optimizer op per parameter; the state tensors are the optimizer's own
    accumulators (created if the optimizer has not stepped yet), saved as persistables"""
    from .serialize import _set_attr
    opt = op.attrs["optimizer"]
    kind = type(opt).__name__.lower()
    kind = kind[:-len("optimizer")] if kind.endswith("optimizer") else kind
    if kind not in ("sgd", "momentum", "adam", "adamw"):
        raise NotImplementedError(f"training program: optimizer {type(opt).__name__} has no reference op here")
    found_inf = op.kwargs.get("found_inf")   # AMP: the optimizer ops read it as SkipUpdate
    grads = _clip_and_decay(w, opt, kind, list(op.kwargs["params"]), list(op.kwargs["grads"]), block_msg)
    lr_val = float(opt.get_lr()) if hasattr(opt, "get_lr") else 0.01
    cache = w.__dict__.setdefault("_lr_tensor", {})
    lr = cache.get(lr_val)
    if lr is None:
        lr = cache[lr_val] = _named(_wrap(torch.tensor([lr_val], dtype=torch.float32)),
                                    f"learning_rate_{len(cache)}")
    for p, g in zip(op.kwargs["params"], grads):
        msg = block_msg.ops.add()
        ins = {"Param": [w.tensor_name(p)], "Grad": [w.tensor_name(g)], "LearningRate": [w.tensor_name(lr)]}
        outs = {"ParamOut": [w.tensor_name(p)]}
        if kind == "sgd":
            msg.type = "sgd"
        elif kind == "momentum":
            msg.type = "momentum"
            vel = opt._acc("velocity", p)
            ins["Velocity"] = outs["VelocityOut"] = [w.tensor_name(_named(vel, vel.name))]
            _set_attr(msg, "mu", float(getattr(opt, "_momentum", 0.9)))
            _set_attr(msg, "use_nesterov", bool(getattr(opt, "_use_nesterov", False)))
        else:
            msg.type = kind
            b1, b2 = float(getattr(opt, "_beta1", 0.9)), float(getattr(opt, "_beta2", 0.999))
            accs = {"Moment1": opt._acc("moment1", p), "Moment2": opt._acc("moment2", p),
                    "Beta1Pow": opt._acc("beta1_pow_acc", p, fill=b1, shape=[1]),
                    "Beta2Pow": opt._acc("beta2_pow_acc", p, fill=b2, shape=[1])}
            for slot, t in accs.items():
                ins[slot] = [w.tensor_name(_named(t, t.name))]
                outs[slot + "Out"] = ins[slot]
            _set_attr(msg, "beta1", b1)
            _set_attr(msg, "beta2", b2)
            _set_attr(msg, "epsilon", float(getattr(opt, "_epsilon", 1e-8)))
            if kind == "adamw":
                coeff = getattr(opt, "_coeff", None)
                if coeff is None:
                    coeff = getattr(opt, "_weight_decay", 0.01)
                _set_attr(msg, "coeff", float(coeff if isinstance(coeff, (int, float)) else 0.01))
                # per parameter, as AdamW._decay_for / _lr_ratio apply them (reference adamw op:
                # with_decay from apply_decay_param_fun, lr_ratio from the lr_ratio callable)
                fn = getattr(opt, "_apply_decay_param_fun", None)
                _set_attr(msg, "with_decay", bool(fn is None or fn(p.name)))
                ratio_fn = getattr(opt, "_lr_ratio_fn", None)
                if ratio_fn is not None:
                    _set_attr(msg, "lr_ratio", float(ratio_fn(p)))
        _set_attr(msg, "op_role", 2)
        if found_inf is not None:
            ins["SkipUpdate"] = [w.tensor_name(found_inf)]
        for slot, names in ins.items():
            v = msg.inputs.add()
            v.parameter = slot
            v.arguments.extend(names)
        for slot, names in outs.items():
            v = msg.outputs.add()
            v.parameter = slot
            v.arguments.extend(names)


def emit_composite_grad(w, program, op, block_msg):
    """the grad op of a call written as several reference ops (static/ref_emit.py COMPOSITE): the
    parts' <type>_grad ops in reverse order, intermediate gradients as ``<name>@GRAD`` variables;
    False when the forward call is not a composite"""
    from . import ref_emit
    from .serialize import _qual_short
    fop = program.__dict__["_grad_of"][id(op)]
    parts = ref_emit.composite(w, _qual_short(fop.type), fop)
    if parts is None:
        return False
    grads = {id(o): g for o, g in zip(op.kwargs["outs"], op.kwargs["gouts"]) if g is not None}
    want = {id(v): g for v, g in zip(op.kwargs["ins"], op.outputs)}
    inter = {id(v) for _, _, outs, _ in parts for vs in outs.values() for v in vs} - \
        {id(v) for v in _tensors(fop.outputs)}
    gparts = []
    for typ, ins, outs, attrs in reversed(parts):
        g_ins = {slot: list(ts) for slot, ts in ins.items()}
        for slot, vs in outs.items():
            g_ins[slot] = list(vs)
            gs = [grads[id(v)] for v in vs if id(v) in grads]
            if gs:
                g_ins[slot + "@GRAD"] = gs
        g_outs = {}
        for slot, ts in ins.items():
            for t in ts:
                if id(t) in want:
                    g_outs.setdefault(slot + "@GRAD", []).append(want[id(t)])
                elif id(t) in inter:
                    gv = ref_emit._tmp_var(t.name + "@GRAD", t, list(t.declared_shape or t.shape))
                    grads[id(t)] = gv
                    g_outs.setdefault(slot + "@GRAD", []).append(gv)
        if g_outs:
            gparts.append((typ + "_grad", g_ins, g_outs, attrs))
    ref_emit.write_parts(w, gparts, block_msg, role=1)
    return True


def _clip_and_decay(w, opt, kind, params, grads, block_msg):
    """the reference's gradient clip (clip.py append_gradient_clip_ops: ClipGradByGlobalNorm as
    squared_l2_norm / sum / sqrt / elementwise_max / elementwise_div / elementwise_mul, ClipGradByValue
    as clip) and L2 regularization (regularizer.py append_regularization_ops: scale + sum) ops in
    front of the optimizer ops; -> the gradients the optimizer ops read"""
    import torch
    from . import ref_emit
    from ..nn.clip import ClipGradByGlobalNorm, ClipGradByValue
    from ..regularizer import L2Decay, L1Decay
    parts = []
    tmp = ref_emit._tmp_var
    clip = getattr(opt, "_grad_clip", None)
    out = list(grads)
    clipped = [i for i, p in enumerate(params) if getattr(p, "need_clip", True)]
    if isinstance(clip, ClipGradByGlobalNorm) and clipped:
        sq = []
        for i in clipped:
            v = tmp(f"{w.tensor_name(grads[i])}@SQ", grads[i], [1], torch.float32)
            parts.append(("squared_l2_norm", {"X": [grads[i]]}, {"Out": [v]}, {}))
            sq.append(v)
        like = sq[0]
        gsq, gn, mx, den, sc = (tmp(f"@CLIP@{opt.__class__.__name__}@{n}", like, [1], torch.float32)
                                for n in ("sum", "norm", "max", "denom", "scale"))
        parts += [("sum", {"X": sq}, {"Out": [gsq]}, {}),
                  ("sqrt", {"X": [gsq]}, {"Out": [gn]}, {}),
                  ("fill_constant", {}, {"Out": [mx]}, {"shape": [1], "value": float(clip.clip_norm),
                                                        "dtype": pb.vartype_of(torch.float32)}),
                  ("elementwise_max", {"X": [gn], "Y": [mx]}, {"Out": [den]}, {"axis": -1}),
                  ("elementwise_div", {"X": [mx], "Y": [den]}, {"Out": [sc]}, {"axis": -1})]
        for i in clipped:
            g = grads[i]
            v = tmp(f"{w.tensor_name(g)}@CLIP", g, list(getattr(g, "declared_shape", None) or g.shape))
            parts.append(("elementwise_mul", {"X": [g], "Y": [sc]}, {"Out": [v]}, {"axis": -1}))
            out[i] = v
    elif isinstance(clip, ClipGradByValue):
        for i in clipped:
            g = out[i]
            v = tmp(f"{w.tensor_name(g)}@CLIP", g, list(getattr(g, "declared_shape", None) or g.shape))
            parts.append(("clip", {"X": [g]}, {"Out": [v]}, {"min": float(clip.min), "max": float(clip.max)}))
            out[i] = v
    elif clip is not None:
        raise NotImplementedError(f"training program: gradient clip {type(clip).__name__} is not written here")
    if kind != "adamw":   # AdamW's decoupled decay is the op's coeff attribute
        for i, p in enumerate(params):
            reg = p.regularizer if getattr(p, "regularizer", None) is not None else getattr(opt, "regularization", None)
            if reg is None:
                continue
            if isinstance(reg, L1Decay) or not isinstance(reg, (L2Decay, int, float)):
                raise NotImplementedError(f"training program: regularizer {type(reg).__name__} is not written here")
            coeff = float(reg.coeff if isinstance(reg, L2Decay) else reg)
            if not coeff:
                continue
            g = out[i]
            shape = list(getattr(g, "declared_shape", None) or g.shape)
            d = tmp(f"{w.tensor_name(p)}@DECAY", g, shape)
            v = tmp(f"{w.tensor_name(g)}@REG", g, shape)
            parts += [("scale", {"X": [p]}, {"Out": [d]}, {"scale": coeff, "bias": 0.0, "bias_after_scale": True}),
                      ("sum", {"X": [g, d]}, {"Out": [v]}, {})]
            out[i] = v
    if parts:
        ref_emit.write_parts(w, parts, block_msg, role=2)
    return out


# ------------------------------------------------------------------------------- AMP loss scaling
def is_amp_op(op):
    from . import passes
    return op.fn in (passes._scaled_ones, passes._unscale_check, passes._update_scaling)


def emit_amp(w, op, msg, ins, outs):
    """static AMP (static/passes.py insert_loss_scaling) as the reference's ops: the loss gradient
    = fill_constant(1) * loss_scaling (elementwise_mul), check_finite_and_unscale (X, Scale -> Out,
    FoundInfinite) and update_loss_scaling (X, FoundInfinite, PrevLossScaling, In{Good,Bad}Steps ->
    Out, LossScaling, Out{Good,Bad}Steps); the optimizer ops then take FoundInfinite as SkipUpdate"""
    from .serialize import _set_attr
    from . import passes, ref_emit
    import torch
    if op.fn is passes._scaled_ones:
        x, scale = op.kwargs["x"], op.kwargs["scale"]
        _named(scale, "loss_scaling_0")
        one = ref_emit._tmp_var(w.tensor_name(op.outputs) + "@ONE", x, list(x._t.shape) or [1])
        msg.type = "fill_constant"
        outs["Out"] = [w.tensor_name(one)]
        _set_attr(msg, "shape", [int(s) for s in (x._t.shape or [1])])
        _set_attr(msg, "value", 1.0)
        _set_attr(msg, "dtype", pb.vartype_of(x._t.dtype))
        _set_attr(msg, "op_role", 257)
        w._pending_parts = [("elementwise_mul", {"X": [one], "Y": [scale]}, {"Out": [op.outputs]},
                             {"axis": -1, "op_role": 257})]
        return
    if op.fn is passes._unscale_check:
        grads, scale = op.kwargs["grads"], op.kwargs["scale"]
        _named(scale, "loss_scaling_0")
        res = list(op.outputs)
        msg.type = "check_finite_and_unscale"
        ins["X"] = [w.tensor_name(g) for g in grads]
        ins["Scale"] = [w.tensor_name(scale)]
        outs["Out"] = [w.tensor_name(v) for v in res[:-1]]
        outs["FoundInfinite"] = [w.tensor_name(res[-1])]
        w._amp_unscaled = res[:-1]
        _set_attr(msg, "op_role", 1)
        return
    kw = op.kwargs
    for t, n in ((kw["scale"], "loss_scaling_0"), (kw["good"], "num_good_steps_0"), (kw["bad"], "num_bad_steps_0")):
        _named(t, n)
    xs = getattr(w, "_amp_unscaled", [])
    msg.type = "update_loss_scaling"
    ins["X"] = [w.tensor_name(v) for v in xs]
    ins["FoundInfinite"] = [w.tensor_name(kw["found_inf"])]
    ins["PrevLossScaling"] = [w.tensor_name(kw["scale"])]
    ins["InGoodSteps"] = [w.tensor_name(kw["good"])]
    ins["InBadSteps"] = [w.tensor_name(kw["bad"])]
    outs["Out"] = list(ins["X"])
    outs["LossScaling"] = list(ins["PrevLossScaling"])
    outs["OutGoodSteps"] = list(ins["InGoodSteps"])
    outs["OutBadSteps"] = list(ins["InBadSteps"])
    for a in ("incr_every", "decr_every"):
        pass
    _set_attr(msg, "incr_every_n_steps", int(kw["incr_every"]))
    _set_attr(msg, "decr_every_n_nan_or_inf", int(kw["decr_every"]))
    _set_attr(msg, "incr_ratio", float(kw["incr_ratio"]))
    _set_attr(msg, "decr_ratio", float(kw["decr_ratio"]))
    _set_attr(msg, "stop_update", False)
    _set_attr(msg, "op_role", 2)
    _ = torch
