"""Per-op backward for the static Program (reference: python/paddle/fluid/backward.py:1141
``_append_backward_ops_``, :1381 ``append_backward``, :1555 ``_append_backward_vars_``; the grad-op
makers of paddle/fluid/framework/grad_op_desc_maker.h).

``append_backward(loss)`` walks the forward ops of the global block in reverse and appends, for
every op on a path from a trainable parameter (or a ``stop_gradient=False`` input) to ``loss``,
ONE grad OpDesc of type ``<forward type>_grad``:

    inputs   the forward op's inputs and outputs and the outputs' ``@GRAD`` Variables
    outputs  ``<input>@GRAD`` for every input that needs a gradient

preceded by a ``fill_constant`` op producing ``loss@GRAD`` (ones), and a ``sum`` op wherever a
Variable feeds several ops (the contributions are named ``x@GRAD@RENAME@<k>`` as in the
reference and summed into ``x@GRAD`` right before the first grad op that reads it). Every appended
op carries ``attrs["op_role"] = "backward"`` and ``attrs["op_role_var"]`` (reference OpRole).

Kernel of a grad op: the vector-Jacobian product of ITS forward op, ``torch.autograd.grad`` from the
forward op's output values to its input values with the output gradients — the executor runs the
forward ops on the autograd tape, so the grad op differentiates exactly that op's recorded
computation (no recomputation, no whole-graph closure). Because the backward is an op list, program
passes can see and rewrite it: static recompute re-runs forward segments inside grad ops, AMP
casts grads, the DP optimizer inserts each all-reduce right after the last grad op of its bucket
(parallel/fleet/static_optimizers.py).
"""
from __future__ import annotations

import torch

from ..framework.core import Tensor, _wrap
from . import program as P

BACKWARD, OPTIMIZE, FORWARD, LOSS = "backward", "optimize", "forward", "loss"


def op_role(op):
    r = op.attrs.get("op_role")
    if r is not None:
        return r
    return BACKWARD if op.type in ("@backward", "@gradients") else (
        OPTIMIZE if op.type in ("@optimize", "@update") else FORWARD)


def is_forward(op):
    return op_role(op) == FORWARD


# ----------------------------------------------------------------------------- grad kernels
def _vjp(outs, ins, gouts):
    """d(ins) of one forward op from its outputs' gradients"""
    o_t, g_t = [], []
    for o, g in zip(outs, gouts):
        if o is None or g is None:
            continue
        t = o._t if isinstance(o, Tensor) else o
        if not (isinstance(t, torch.Tensor) and t.requires_grad):
            continue
        gt = g._t if isinstance(g, Tensor) else g
        o_t.append(t)
        g_t.append(gt.to(t.dtype) if gt.dtype != t.dtype else gt)
    in_t = [i._t if isinstance(i, Tensor) else i for i in ins]
    req = [k for k, t in enumerate(in_t) if isinstance(t, torch.Tensor) and t.requires_grad]
    res = [None] * len(in_t)
    if o_t and req:
        gs = torch.autograd.grad(o_t, [in_t[k] for k in req], g_t, allow_unused=True, retain_graph=True)
        for k, g in zip(req, gs):
            res[k] = g
    return tuple(_wrap(r if r is not None else torch.zeros_like(t)) for r, t in zip(res, in_t))


def _fill_ones(x):
    return _wrap(torch.ones_like(x._t))


def _sum(xs):
    acc = xs[0]._t
    for x in xs[1:]:
        acc = acc + x._t
    return _wrap(acc)


# ----------------------------------------------------------------------------- program rewriting
def _sub_block_ops(program, op):
    for k in P._SUB_BLOCK_ATTRS:
        b = op.attrs.get(k)
        if isinstance(b, int) and 0 <= b < len(program.blocks):
            for sop in program.blocks[b].ops:
                yield sop
                yield from _sub_block_ops(program, sop)


def _op_inputs(program, op):
    """the Variables and Parameters an op reads, including what a control-flow op's sub-blocks
    capture from the enclosing block"""
    seen, out = set(), []

    def add(v):
        if id(v) not in seen:
            seen.add(id(v))
            out.append(v)
    for v in P._iter_tensors((op.args, op.kwargs, list(op.attrs.get("captured", [])))):
        add(v)
    if op.exec is not None:
        ids = P._op_uses(program, op)
        blk0 = program.global_block()
        for v in blk0.vars.values():
            if id(v) in ids:
                add(v)
        for sop in _sub_block_ops(program, op):
            for v in P._iter_tensors((sop.args, sop.kwargs)):
                if isinstance(v, P.Parameter):
                    add(v)
    return out


def _floating(v):
    t = getattr(v, "_t", None)
    return isinstance(t, torch.Tensor) and (t.is_floating_point() or t.is_complex())


def _grad_type(op):
    base = op.type.rsplit(".", 1)[-1] if op.type.startswith("paddle_hackathon_amd.") else op.type
    return base + "_grad"


def _new_grad_var(blk, like, name):
    if name in blk.vars:
        return blk.vars[name]
    return P._grad_var(blk, like, name)


def append_backward_ops(targets, target_grads=None, sources=None, no_grad_set=None, program=None):
    """Append the grad ops of ``targets`` (list of Variables) and return {id(source): grad Variable}
    for ``sources`` (Variables / Parameters; default: every trainable parameter)."""
    prog = program or P.default_main_program()
    blk = prog.global_block()
    fwd_ops = [op for op in blk.ops if is_forward(op)]
    nog = {id(v) for v in (no_grad_set or []) if not isinstance(v, str)}
    nog_names = {v for v in (no_grad_set or []) if isinstance(v, str)}

    def blocked(v):
        return id(v) in nog or getattr(v, "name", None) in nog_names

    if sources is None:
        sources = [p for p in prog.all_parameters() if p.trainable]
    # 1. which Variables carry gradient (forward propagation from the sources / need_grad inputs)
    req = {id(s) for s in sources if not blocked(s)}
    for v in blk.vars.values():
        if isinstance(v, P.Variable) and getattr(v, "need_grad", False) and _floating(v) and not blocked(v):
            req.add(id(v))
    for op in fwd_ops:
        if any(id(v) in req for v in _op_inputs(prog, op)):
            for o in P._iter_vars(op.outputs):
                if _floating(o) and not blocked(o):
                    req.add(id(o))
    # 2. ops on a path to the targets
    needed = {id(t) for t in targets}
    path = []
    for op in reversed(fwd_ops):
        if any(id(o) in needed for o in P._iter_vars(op.outputs)):
            path.append(op)
            for v in _op_inputs(prog, op):
                if id(v) in req:
                    needed.add(id(v))
    # how many gradient contributions each Variable will receive: with more than one, every
    # contribution is a @RENAME@ Variable and a sum op forms <name>@GRAD (reference
    # _addup_repetitive_outputs_)
    n_contrib = {}
    for t in targets:
        n_contrib[id(t)] = n_contrib.get(id(t), 0) + 1
    for op in path:
        for v in _op_inputs(prog, op):
            if id(v) in req and id(v) in needed:
                n_contrib[id(v)] = n_contrib.get(id(v), 0) + 1
    # 3. emit
    contrib = {}   # id(var) -> [grad Variables]
    var_of = {}
    final = {}     # id(var) -> the summed grad Variable

    def add_contrib(v, g):
        contrib.setdefault(id(v), []).append(g)
        var_of[id(v)] = v

    def finalize(v):
        """the grad Variable of v, summing the contributions first if several"""
        vid = id(v)
        if vid in final:
            return final[vid]
        cs = contrib.get(vid)
        if not cs:
            return None
        if len(cs) == 1:
            g = cs[0]
        else:
            g = _new_grad_var(blk, v, v.name + "@GRAD")
            op = P.OpDesc("sum", _sum, (), {"xs": tuple(cs)}, g,
                          attrs={"op_role": BACKWARD, "op_role_var": [v.name]})
            g.op = op
            blk.append_op(op)
        final[vid] = g
        return g

    for t, tg in zip(targets, target_grads or [None] * len(targets)):
        if tg is None:
            g = _new_grad_var(blk, t, t.name + "@GRAD")
            op = P.OpDesc("fill_constant", _fill_ones, (), {"x": t}, g,
                          attrs={"op_role": LOSS, "value": 1.0, "op_role_var": [t.name]})
            g.op = op
            blk.append_op(op)
        else:
            g = tg
        add_contrib(t, g)
    counter = [0]
    for op in path:
        outs = list(P._iter_vars(op.outputs))
        gouts = [finalize(o) if id(o) in contrib else None for o in outs]
        if all(g is None for g in gouts):
            continue
        ins = [v for v in _op_inputs(prog, op) if id(v) in req and id(v) in needed]
        if not ins:
            continue
        gins = []
        for v in ins:
            nm = v.name + "@GRAD"
            if n_contrib.get(id(v), 0) > 1 or nm in blk.vars:
                counter[0] += 1
                nm = f"{v.name}@GRAD@RENAME@block0@{counter[0]}"
            gins.append(_new_grad_var(blk, v, nm))
        gop = P.OpDesc(_grad_type(op), _vjp, (), {"outs": tuple(outs), "ins": tuple(ins), "gouts": tuple(gouts)},
                       tuple(gins), attrs={"op_role": BACKWARD, "fwd_type": op.type, "_fwd_id": id(op),
                                           "op_role_var": [v.name for v in ins]})
        prog.__dict__.setdefault("_cut_ops", set()).add(id(op))
        for g in gins:
            g.op = gop
        blk.append_op(gop)
        prog.__dict__.setdefault("_grad_of", {})[id(gop)] = op   # for passes (recompute)
        for v, g in zip(ins, gins):
            add_contrib(v, g)
    res = {}
    for s in sources:
        g = finalize(s) if id(s) in contrib else None
        if g is not None and g.name != s.name + "@GRAD" and (s.name + "@GRAD") not in blk.vars:
            # a lone renamed contribution: give the parameter its canonical @GRAD name
            alias = _new_grad_var(blk, s, s.name + "@GRAD")
            op = P.OpDesc("assign", lambda x: _wrap(x._t), (), {"x": g}, alias,
                          attrs={"op_role": BACKWARD, "op_role_var": [s.name]})
            alias.op = op
            blk.append_op(op)
            g = alias
        res[id(s)] = g
    return res


def append_backward(loss, parameter_list=None, no_grad_set=None, callbacks=None, checkpoints=None,
                    distop_context=None):
    """reference ``paddle.static.append_backward``: [(param, param@GRAD)] with per-op grad ops"""
    prog = P.default_main_program()
    blk = prog.global_block()
    params = parameter_list if parameter_list is not None else [p for p in prog.all_parameters() if p.trainable]
    params = [blk.vars.get(p, p) if isinstance(p, str) else p for p in params]
    nog = set(id(v) for v in (no_grad_set or []) if not isinstance(v, str))
    params = [p for p in params if id(p) not in nog]
    if checkpoints:
        from .passes import recompute_segments
        prog.__dict__["_recompute_checkpoints"] = list(checkpoints)
    grads = append_backward_ops([loss], sources=params, no_grad_set=no_grad_set, program=prog)
    out = []
    for p in params:
        g = grads.get(id(p))
        if g is None:   # not on a path to the loss: a zero gradient, as the reference fills
            g = _new_grad_var(blk, p, p.name + "@GRAD")
            op = P.OpDesc("fill_zeros_like", lambda x: _wrap(torch.zeros_like(x._t)), (), {"x": p}, g,
                          attrs={"op_role": BACKWARD, "op_role_var": [p.name]})
            g.op = op
            blk.append_op(op)
        out.append((p, g))
    if checkpoints:
        recompute_segments(prog, checkpoints)
    return out


def gradients(targets, inputs, target_gradients=None, no_grad_set=None):
    """reference ``paddle.static.gradients``: grad Variables of ``inputs`` (per-op grad ops)"""
    prog = P.default_main_program()
    targets = [targets] if isinstance(targets, Tensor) else list(targets)
    inputs = [inputs] if isinstance(inputs, Tensor) else list(inputs)
    for v in inputs:
        if isinstance(v, P.Variable):
            v.need_grad = True
    tg = target_gradients if target_gradients is None or isinstance(target_gradients, (list, tuple)) \
        else [target_gradients]
    grads = append_backward_ops(targets, tg, sources=inputs, no_grad_set=no_grad_set, program=prog)
    blk = prog.global_block()
    out = []
    for x in inputs:
        g = grads.get(id(x))
        if g is None:
            g = _new_grad_var(blk, x, x.name + "@GRAD")
            op = P.OpDesc("fill_zeros_like", lambda v: _wrap(torch.zeros_like(v._t)), (), {"x": x}, g,
                          attrs={"op_role": BACKWARD})
            g.op = op
            blk.append_op(op)
        out.append(g)
    return out


def append_optimize_op(optimizer, params_grads, program=None, block=None, found_inf=None):
    """one fused optimizer op over (param, grad) pairs (reference: the per-parameter optimizer ops
    fused by fuse_optimizer_ops_pass); type = the optimizer's name (``adamw``, ``momentum`` ...).
    found_inf (AMP): a bool Variable; the update is skipped on the steps where it is true (the
    reference's optimizer ops read it as their SkipUpdate input)."""
    prog = program or P.default_main_program()
    blk = block or prog.current_block()
    ps = tuple(p for p, _ in params_grads)
    gs = tuple(g for _, g in params_grads)
    if optimizer._parameter_list is None:
        optimizer._add_param_group({"params": list(ps)})
        optimizer._parameter_list = list(ps)

    def _update(params, grads, found_inf=None):
        if found_inf is not None and bool(found_inf._t):
            return None
        # in a non-root Scope the params are that scope's copies: step them with its own state;
        # Hogwild dataset-trainer threads apply their updates one at a time
        from .trainer import hogwild_update
        # lock-free Hogwild batches ran on parameter aliases: the update goes to the real ones
        params = [getattr(p, "_hogwild_of", p) for p in params]
        with hogwild_update(), P.optimizer_lock(optimizer), P.scoped_optimizer(optimizer, ps, params):
            for p, g in zip(params, grads):
                p._t.grad = g._t.detach().to(p._t.dtype)
            with P._core_dynamic():
                optimizer.step()
            optimizer.clear_grad(set_to_zero=False)
        return None

    kw = {"params": ps, "grads": gs}
    if found_inf is not None:
        kw["found_inf"] = found_inf
    op = P.OpDesc(type(optimizer).__name__.lower(), _update, (), kw, None,
                  attrs={"op_role": OPTIMIZE, "op_role_var": [p.name for p in ps], "optimizer": optimizer})
    blk.append_op(op)
    return op


def minimize(optimizer, loss, parameters=None, no_grad_set=None):
    """static ``optimizer.minimize``: per-op backward + one optimizer op"""
    prog = P.default_main_program()
    params = parameters if parameters is not None else [p for p in prog.all_parameters() if p.trainable]
    nog = set(id(v) for v in (no_grad_set or []) if not isinstance(v, str))
    params = [p for p in params if id(p) not in nog]
    if optimizer._parameter_list is None:
        optimizer._add_param_group({"params": list(params)})
        optimizer._parameter_list = list(params)
    pg = append_backward(loss, params, no_grad_set)
    op = append_optimize_op(optimizer, pg, prog)
    return [op], pg
