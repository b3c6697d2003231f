"""Backward and optimizer ops of reference-written TRAINING ProgramDescs (reference:
paddle/fluid/operators/*_op.cc GradOpMaker outputs — ``<type>_grad`` ops with the forward's input
slots, ``<Out>@GRAD`` inputs and ``<X>@GRAD`` outputs; optimizers/{sgd,momentum,adam,adamw,
adagrad,rmsprop}_op.cc with Param / Grad / LearningRate / moment slots and in-place ``*Out``).

A generic ``<type>_grad`` converter rebuilds the forward op from its input slots with the
forward converter of static/ref_ops.py, re-runs it on autograd leaves and takes the vector-Jacobian
product against the ``@GRAD`` inputs (recompute, as a reference grad kernel reads the forward's
inputs). Grad ops whose maker passes the forward OUTPUT instead of the input (relu / sigmoid /
tanh / exp / sqrt / softmax ..., softmax_with_cross_entropy's Softmax) have closed forms here.
Optimizer ops update the persistable parameter and state tensors in place, so a loaded training
program steps exactly like the reference executor runs it."""
from __future__ import annotations

import torch

from ..framework.core import Tensor, _wrap

__all__ = ["grad_converter", "OPTIMIZERS"]


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def _leafs(tree, targets):
    """tensors of ``tree`` (nested lists / dicts of Tensors) as detached fp leaves; the target
    positions (ids of the original Tensor objects) require grad"""
    made = {}

    def conv(v):
        if isinstance(v, Tensor):
            t = v._t.detach()
            if id(v) in targets and t.is_floating_point():
                t = t.clone().requires_grad_(True)
                made[id(v)] = t
            return _wrap(t)
        if isinstance(v, (list, tuple)):
            return type(v)(conv(e) for e in v)
        if isinstance(v, dict):
            return {k: conv(e) for k, e in v.items()}
        return v
    return conv(tree), made


def recompute_vjp(fwd_fn, fwd_kwargs, targets, douts):
    """d(sum_i <fwd outputs_i, douts_i>) / d targets; None for targets without a path"""
    ids = {id(t): i for i, t in enumerate(targets) if t is not None}
    kw, made = _leafs(fwd_kwargs, ids)
    with torch.enable_grad():
        out = fwd_fn(**kw)
    outs = list(out) if isinstance(out, (list, tuple)) else [out]
    pairs = [(_t(o), _t(g)) for o, g in zip(outs, douts) if g is not None and o is not None and _t(o).requires_grad]
    leaves = [made.get(id(t)) if t is not None else None for t in targets]
    live = [l for l in leaves if l is not None]
    res = [None] * len(targets)
    if pairs and live:
        gs = torch.autograd.grad([o for o, _ in pairs], live, [g.to(o.dtype).reshape(o.shape) for o, g in pairs],
                                 allow_unused=True)
        it = iter(gs)
        for i, l in enumerate(leaves):
            if l is not None:
                g = next(it)
                res[i] = _wrap(g if g is not None else torch.zeros_like(l))
    seen = set()
    for i, t in enumerate(targets):   # an input at several positions: its whole gradient once (the
        if t is not None and id(t) in seen and res[i] is not None:   # writer sums the positions)
            res[i] = _wrap(torch.zeros_like(_t(res[i])))
        if t is not None:
            seen.add(id(t))
    for i, t in enumerate(targets):   # integer inputs / unused: zeros of the input's shape
        if res[i] is None and t is not None:
            res[i] = _wrap(torch.zeros_like(_t(t), dtype=_t(t).dtype if _t(t).is_floating_point() else torch.float32))
    return tuple(res)


def ref_grad_op(fwd_fn, fwd_kwargs, targets, douts):
    """the recorded grad op: one gradient per ``targets`` entry"""
    return recompute_vjp(fwd_fn, fwd_kwargs, list(targets), list(douts))


# ---------------------------------------------------------------- grads from the forward output
def _out_based(kind):
    def fn(out, dout, **at):
        o, g = _t(out).float(), _t(dout).float()
        if kind == "relu":
            r = g * (o > 0)
        elif kind == "relu6":
            r = g * ((o > 0) & (o < at.get("threshold", 6.0)))
        elif kind == "sigmoid":
            r = g * o * (1 - o)
        elif kind == "tanh":
            r = g * (1 - o * o)
        elif kind == "exp":
            r = g * o
        elif kind == "sqrt":
            r = g * 0.5 / o
        elif kind == "rsqrt":
            r = g * -0.5 * o * o * o
        elif kind == "reciprocal":
            r = g * -(o * o)
        elif kind == "softmax":
            ax = at.get("axis", -1)
            r = o * (g - (g * o).sum(ax, keepdim=True))
        elif kind == "log_softmax":
            ax = at.get("axis", -1)
            r = g - torch.exp(o) * g.sum(ax, keepdim=True)
        else:
            raise NotImplementedError(kind)
        return _wrap(r.to(_t(dout).dtype))
    return fn


_OUT_BASED = {"relu", "relu6", "sigmoid", "tanh", "exp", "sqrt", "rsqrt", "reciprocal", "softmax", "log_softmax"}


def softmax_ce_grad(softmax, label, loss_grad, soft_label=False, ignore_index=-100, axis=-1):
    """softmax_with_cross_entropy_grad: dLogits = (softmax - onehot(label)) * dLoss"""
    p = _t(softmax).float()
    ax = axis % p.dim()
    g = _t(loss_grad).float()
    if soft_label:
        d = p - _t(label).float()
    else:
        lab = _t(label).long()
        if lab.dim() == p.dim():
            lab = lab.squeeze(ax)
        keep = lab != ignore_index
        oh = torch.nn.functional.one_hot(lab.clamp_min(0), p.shape[ax]).to(p.dtype).movedim(-1, ax)
        d = (p - oh) * keep.unsqueeze(ax)
    return _wrap((d * g).to(_t(softmax).dtype))


def softmax_ce_op(logits, label, soft_label=False, ignore_index=-100, axis=-1):
    """softmax_with_cross_entropy (forward): (Softmax, Loss) with Loss keeping the class axis as 1"""
    x = _t(logits)
    ax = axis % x.dim()
    logp = torch.log_softmax(x.float(), ax)
    if soft_label:
        loss = -(_t(label).float() * logp).sum(ax, keepdim=True)
    else:
        lab = _t(label).long()
        if lab.dim() == x.dim():
            lab = lab.squeeze(ax)
        keep = lab != ignore_index
        loss = -logp.gather(ax, lab.clamp_min(0).unsqueeze(ax)) * keep.unsqueeze(ax)
    return _wrap(logp.exp().to(x.dtype)), _wrap(loss.to(x.dtype))


def _conv_swce(r, ins, at):
    return softmax_ce_op, {"logits": _one(r, ins, "Logits"), "label": _one(r, ins, "Label"),
                           "soft_label": at.get("soft_label", False), "ignore_index": at.get("ignore_index", -100),
                           "axis": at.get("axis", -1)}, ("Softmax", "Loss")


FORWARD = {"softmax_with_cross_entropy": _conv_swce}
# (AMP converters registered below, with the optimizers)


def _align(y, xdim, axis):
    """y's shape placed into x's rank by the reference rule (Y's dims start at ``axis``)"""
    yr = y.dim()
    if axis in (-1, None) or yr >= xdim:
        return y.reshape([1] * (xdim - yr) + list(y.shape))
    return y.reshape([1] * axis + list(y.shape) + [1] * (xdim - axis - yr))


def _reduce_to(g, shape_aligned, shape):
    dims = [i for i, (a, b) in enumerate(zip(g.shape, shape_aligned)) if b == 1 and a != 1]
    if dims:
        g = g.sum(dims, keepdim=True)
    return g.reshape(shape)


def elementwise_grad(kind, x, y, dout, axis=-1, want=("X@GRAD", "Y@GRAD")):
    """elementwise_{add,sub,mul,div,max,min}_grad with the reference's axis broadcasting"""
    xt, yt, g = _t(x), _t(y), _t(dout).float()
    nd = max(xt.dim(), yt.dim())
    xa = _align(xt, nd, -1) if xt.dim() < nd else xt
    ya = _align(yt, nd, axis) if yt.dim() < nd else yt
    xf, yf = xa.float(), ya.float()
    if kind == "add":
        dx, dy = g, g
    elif kind == "sub":
        dx, dy = g, -g
    elif kind == "mul":
        dx, dy = g * yf, g * xf
    elif kind == "div":
        dx, dy = g / yf, -g * xf / (yf * yf)
    elif kind in ("max", "min"):
        m = (xf > yf) if kind == "max" else (xf < yf)
        dx, dy = g * m, g * (~m)
    else:
        raise NotImplementedError(kind)
    outs = {"X@GRAD": _wrap(_reduce_to(dx.expand(g.shape), xa.shape, xt.shape).to(xt.dtype)),
            "Y@GRAD": _wrap(_reduce_to(dy.expand(g.shape), ya.shape, yt.shape).to(yt.dtype))}
    res = tuple(outs[w] for w in want)
    return res if len(res) > 1 else res[0]


def reshape_grad(dout, x_shape):
    """reshape2 / squeeze2 / unsqueeze2 / flatten2 grads: the output gradient in X's shape (from
    the XShape variable's declared shape [0, *x.shape])"""
    return _wrap(_t(dout).reshape([int(v) for v in x_shape]))


def dropout_grad(dout, mask, p=0.5, implementation="downgrade_in_infer"):
    """dropout_grad: dX = dOut * Mask (/ (1 - p) for upscale_in_train) — the forward's mask, not a
    new draw"""
    g = _t(dout)
    d = g * _t(mask).to(g.dtype)
    if implementation == "upscale_in_train":
        d = d / (1.0 - p) if p < 1.0 else torch.zeros_like(g)
    return _wrap(d)


def reshape_like(dout, x):
    return _wrap(_t(dout).reshape(_t(x).shape))


def transpose_grad(dout, axis):
    inv = [0] * len(axis)
    for i, a in enumerate(axis):
        inv[a] = i
    return _wrap(_t(dout).permute(inv))


_ELT = {f"elementwise_{k}": k for k in ("add", "sub", "mul", "div", "max", "min")}


def grad_converter(fwd_type, convert):
    """the converter of ``<fwd_type>_grad`` (or None): convert = the reader's forward table"""
    if fwd_type in _OUT_BASED:
        def conv(r, ins, at):
            kw = {k: v for k, v in at.items() if k in ("threshold", "axis")}
            return _out_based(fwd_type), dict(out=_one(r, ins, "Out"), dout=_one(r, ins, "Out@GRAD"), **kw), "X@GRAD"
        return conv
    if fwd_type == "softmax_with_cross_entropy":
        def conv(r, ins, at):
            return softmax_ce_grad, {"softmax": _one(r, ins, "Softmax"), "label": _one(r, ins, "Label"),
                                     "loss_grad": _one(r, ins, "Loss@GRAD"), "soft_label": at.get("soft_label", False),
                                     "ignore_index": at.get("ignore_index", -100), "axis": at.get("axis", -1)}, \
                "Logits@GRAD"
        return conv
    if fwd_type in _ELT:
        def conv(r, ins, at):
            want = tuple(r._grad_out_slots)
            return elementwise_grad, {"kind": _ELT[fwd_type], "x": _one(r, ins, "X"), "y": _one(r, ins, "Y"),
                                      "dout": _one(r, ins, "Out@GRAD"), "axis": at.get("axis", -1), "want": want}, \
                (want[0] if len(want) == 1 else want)
        return conv
    if fwd_type in ("reshape2", "squeeze2", "unsqueeze2", "flatten2"):
        def conv(r, ins, at):
            if "XShape" in ins:
                xs = r.var(ins["XShape"][0])
                shape = list(getattr(xs, "declared_shape", None) or xs.shape)[1:]
                return reshape_grad, {"dout": _one(r, ins, "Out@GRAD"), "x_shape": shape}, "X@GRAD"
            # no XShape (a program written here): the grad op carries the forward input X itself
            return reshape_like, {"dout": _one(r, ins, "Out@GRAD"), "x": _one(r, ins, "X")}, "X@GRAD"
        return conv
    if fwd_type == "dropout":
        def conv(r, ins, at):
            return dropout_grad, {"dout": _one(r, ins, "Out@GRAD"), "mask": _one(r, ins, "Mask"),
                                  "p": at.get("dropout_prob", 0.5),
                                  "implementation": at.get("dropout_implementation", "downgrade_in_infer")}, "X@GRAD"
        return conv
    if fwd_type == "transpose2":
        def conv(r, ins, at):
            return transpose_grad, {"dout": _one(r, ins, "Out@GRAD"), "axis": list(at.get("axis", []))}, "X@GRAD"
        return conv
    fwd = convert.get(fwd_type)
    if fwd is None:
        return None

    def conv(r, ins, at):
        fwd_ins = {k: v for k, v in ins.items() if not k.endswith("@GRAD")}
        fn, kwargs, out_spec = fwd(r, fwd_ins, at)
        fn = getattr(fn, "__wrapped_op__", fn)
        # output gradients in the forward's output order
        if isinstance(out_spec, str):
            douts = [_one(r, ins, out_spec + "@GRAD")]
        elif out_spec[0] == "list":
            douts = [r.var(n) for n in ins.get(out_spec[1] + "@GRAD", [])]
        else:
            douts = [_one(r, ins, sl + "@GRAD") for sl in out_spec]
        grad_slots = r._grad_out_slots   # set by the reader: the op's "<slot>@GRAD" outputs, in order
        targets = [_one(r, fwd_ins, sl[:-5]) for sl in grad_slots]
        return ref_grad_op, {"fwd_fn": fn, "fwd_kwargs": kwargs, "targets": targets, "douts": douts}, \
            tuple(grad_slots)
    return conv


def _one(r, ins, slot):
    return r.var(ins[slot][0]) if ins.get(slot) else None


# ------------------------------------------------------------------------------- optimizers
def _lr(lr):
    return float(_t(lr).reshape(-1)[0]) if lr is not None else 0.0


def _decay(g, p, method, coeff):
    if method == "l2_decay" and coeff:
        return g + coeff * p
    return g


def sgd_op(param, grad, learning_rate):
    p = _t(param)
    with torch.no_grad():
        p.sub_(_lr(learning_rate) * _t(grad).to(p.dtype))
    return param


def momentum_op(param, grad, velocity, learning_rate, mu=0.9, use_nesterov=False, regularization_method="",
                regularization_coeff=0.0, rescale_grad=1.0):
    p, v = _t(param), _t(velocity)
    with torch.no_grad():
        g = _decay(_t(grad).float() * rescale_grad, p.float(), regularization_method, regularization_coeff)
        v.mul_(mu).add_(g.to(v.dtype))
        lr = _lr(learning_rate)
        upd = (g + mu * v.float()) if use_nesterov else v.float()
        p.sub_((lr * upd).to(p.dtype))
    return param, velocity


def adam_op(param, grad, learning_rate, moment1, moment2, beta1_pow, beta2_pow, beta1=0.9, beta2=0.999,
            epsilon=1e-8, coeff=0.0, with_decay=False, lr_ratio=1.0):
    """adam_op.cc / adamw_op.cc: lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t) with the pow accumulators
    (Beta1Pow = b1^t before this step's update), eps added to sqrt(m2) scaled as the reference"""
    p, m1, m2, b1p, b2p = (_t(v) for v in (param, moment1, moment2, beta1_pow, beta2_pow))
    with torch.no_grad():
        g = _t(grad).float()
        lr = _lr(learning_rate) * lr_ratio
        if with_decay and coeff:
            p.mul_(1.0 - lr * coeff)
        m1.mul_(beta1).add_((1 - beta1) * g)
        m2.mul_(beta2).add_((1 - beta2) * g * g)
        b1, b2 = float(b1p.reshape(-1)[0]), float(b2p.reshape(-1)[0])
        lr_t = lr * (1 - b2) ** 0.5 / (1 - b1)
        p.sub_((lr_t * m1 / (m2.sqrt() + epsilon * (1 - b2) ** 0.5)).to(p.dtype))
        b1p.mul_(beta1)
        b2p.mul_(beta2)
    return param, moment1, moment2, beta1_pow, beta2_pow


def adagrad_op(param, grad, moment, learning_rate, epsilon=1e-6):
    p, m = _t(param), _t(moment)
    with torch.no_grad():
        g = _t(grad).float()
        m.add_(g * g)
        p.sub_((_lr(learning_rate) * g / (m.sqrt() + epsilon)).to(p.dtype))
    return param, moment


def rmsprop_op(param, grad, moment, mean_square, learning_rate, mean_grad=None, epsilon=1e-10, decay=0.9,
               momentum=0.0, centered=False):
    p, mom, ms = _t(param), _t(moment), _t(mean_square)
    with torch.no_grad():
        g = _t(grad).float()
        ms.mul_(decay).add_((1 - decay) * g * g)
        if centered:
            mg = _t(mean_grad)
            mg.mul_(decay).add_((1 - decay) * g)
            den = (ms - mg * mg + epsilon).sqrt()
        else:
            den = (ms + epsilon).sqrt()
        mom.mul_(momentum).add_(_lr(learning_rate) * g / den)
        p.sub_(mom.to(p.dtype))
    return param, moment, mean_square


def _skipping(fn, returns):
    """the optimizer op with its SkipUpdate input (AMP: the step found inf / nan): no update, the
    state tensors pass through"""
    def run(skip_update=None, **kw):
        if skip_update is not None and bool(_t(skip_update).reshape(-1)[0]):
            res = tuple(kw[k] for k in returns)
            return res if len(res) > 1 else res[0]
        return fn(**kw)
    run.__name__ = fn.__name__
    run.__module__ = fn.__module__
    return run


def _opt_conv(fn, slots, outs, attrs):
    returns = [k for k in slots if k in ("param", "velocity", "moment", "moment1", "moment2", "beta1_pow",
                                         "beta2_pow", "mean_square", "mean_grad")]
    skipping = _skipping(fn, returns)

    def conv(r, ins, at):
        kw = {k: _one(r, ins, s) for k, s in slots.items()}
        kw.update({k: at.get(a, d) for k, (a, d) in attrs.items()})
        if ins.get("SkipUpdate"):
            kw["skip_update"] = _one(r, ins, "SkipUpdate")
            return skipping, kw, tuple(outs)
        return fn, kw, tuple(outs)
    return conv


# ------------------------------------------------------------------------------- AMP loss scaling
def check_finite_unscale_op(xs, scale):
    """check_finite_and_unscale_op.cc: Out = X / Scale, FoundInfinite = any non-finite"""
    inv = 1.0 / _t(scale).float().reshape(-1)[0]
    bad = None
    outs = []
    for x in xs:
        u = _t(x).float() * inv
        b = ~torch.isfinite(u).all()
        bad = b if bad is None else (bad | b)
        outs.append(_wrap(u.to(_t(x).dtype)))
    if bad is None:
        bad = torch.zeros((), dtype=torch.bool)
    return outs, _wrap(bad.reshape(1))


def update_loss_scaling_op(xs, found_inf, prev_scale, good, bad, incr_every_n_steps=1000, decr_every_n_nan_or_inf=2,
                           incr_ratio=2.0, decr_ratio=0.5, stop_update=False):
    """update_loss_scaling_op.cc: on overflow the gradients are zeroed and the bad-step counter
    grows (scale * decr_ratio every decr_every_n_nan_or_inf of them, kept >= 1); otherwise the
    good-step counter grows (scale * incr_ratio every incr_every_n_steps)"""
    with torch.no_grad():
        inf = bool(_t(found_inf).reshape(-1)[0])
        if inf:
            for x in xs:
                _t(x).zero_()
        if not stop_update:
            s, gd, bd = _t(prev_scale), _t(good), _t(bad)
            if inf:
                gd.zero_()
                bd.add_(1)
                if int(bd.reshape(-1)[0]) >= decr_every_n_nan_or_inf:
                    s.mul_(decr_ratio).clamp_(min=1.0)
                    bd.zero_()
            else:
                bd.zero_()
                gd.add_(1)
                if int(gd.reshape(-1)[0]) >= incr_every_n_steps:
                    s.mul_(incr_ratio)
                    gd.zero_()
    return list(xs), prev_scale, good, bad


def _conv_cfu(r, ins, at):
    return check_finite_unscale_op, {"xs": [r.var(n) for n in ins.get("X", [])], "scale": _one(r, ins, "Scale")}, \
        ("Out*", "FoundInfinite")


def _conv_uls(r, ins, at):
    return update_loss_scaling_op, {
        "xs": [r.var(n) for n in ins.get("X", [])], "found_inf": _one(r, ins, "FoundInfinite"),
        "prev_scale": _one(r, ins, "PrevLossScaling"), "good": _one(r, ins, "InGoodSteps"),
        "bad": _one(r, ins, "InBadSteps"), "incr_every_n_steps": at.get("incr_every_n_steps", 1000),
        "decr_every_n_nan_or_inf": at.get("decr_every_n_nan_or_inf", 2), "incr_ratio": at.get("incr_ratio", 2.0),
        "decr_ratio": at.get("decr_ratio", 0.5), "stop_update": at.get("stop_update", False)}, \
        ("Out*", "LossScaling", "OutGoodSteps", "OutBadSteps")


OPTIMIZERS = {
    "sgd": _opt_conv(sgd_op, {"param": "Param", "grad": "Grad", "learning_rate": "LearningRate"}, ["ParamOut"], {}),
    "momentum": _opt_conv(momentum_op, {"param": "Param", "grad": "Grad", "velocity": "Velocity",
                                        "learning_rate": "LearningRate"}, ["ParamOut", "VelocityOut"],
                          {"mu": ("mu", 0.9), "use_nesterov": ("use_nesterov", False),
                           "regularization_method": ("regularization_method", ""),
                           "regularization_coeff": ("regularization_coeff", 0.0),
                           "rescale_grad": ("rescale_grad", 1.0)}),
    "adam": _opt_conv(adam_op, {"param": "Param", "grad": "Grad", "learning_rate": "LearningRate",
                                "moment1": "Moment1", "moment2": "Moment2", "beta1_pow": "Beta1Pow",
                                "beta2_pow": "Beta2Pow"},
                      ["ParamOut", "Moment1Out", "Moment2Out", "Beta1PowOut", "Beta2PowOut"],
                      {"beta1": ("beta1", 0.9), "beta2": ("beta2", 0.999), "epsilon": ("epsilon", 1e-8)}),
    "adamw": _opt_conv(adam_op, {"param": "Param", "grad": "Grad", "learning_rate": "LearningRate",
                                 "moment1": "Moment1", "moment2": "Moment2", "beta1_pow": "Beta1Pow",
                                 "beta2_pow": "Beta2Pow"},
                       ["ParamOut", "Moment1Out", "Moment2Out", "Beta1PowOut", "Beta2PowOut"],
                       {"beta1": ("beta1", 0.9), "beta2": ("beta2", 0.999), "epsilon": ("epsilon", 1e-8),
                        "coeff": ("coeff", 0.01), "with_decay": ("with_decay", True), "lr_ratio": ("lr_ratio", 1.0)}),
    "adagrad": _opt_conv(adagrad_op, {"param": "Param", "grad": "Grad", "moment": "Moment",
                                      "learning_rate": "LearningRate"}, ["ParamOut", "MomentOut"],
                         {"epsilon": ("epsilon", 1e-6)}),
    "rmsprop": _opt_conv(rmsprop_op, {"param": "Param", "grad": "Grad", "moment": "Moment",
                                      "mean_square": "MeanSquare", "learning_rate": "LearningRate",
                                      "mean_grad": "MeanGrad"}, ["ParamOut", "MomentOut", "MeanSquareOut"],
                         {"epsilon": ("epsilon", 1e-10), "decay": ("decay", 0.9), "momentum": ("momentum", 0.0),
                          "centered": ("centered", False)}),
}

FORWARD.update({"check_finite_and_unscale": _conv_cfu, "update_loss_scaling": _conv_uls})
