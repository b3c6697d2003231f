"""Static-graph control flow with sub-blocks (reference: python/paddle/fluid/layers/control_flow.py
``cond`` -> conditional_block ops + select_input, ``while_loop`` -> while op; executor side
paddle/fluid/operators/controlflow/{conditional_block_op,while_op}.cc).

``cond(pred, true_fn, false_fn)`` in static mode records each branch into its own ``Block`` of the
current Program and appends ONE ``conditional_block`` op to the parent block; at run time the
executor evaluates ``pred`` and interprets only the taken branch's block. ``while_loop(cond,
body, loop_vars)`` records the condition and the body against placeholder Variables in two
sub-blocks; the ``while`` op rebinds the placeholders every iteration. Branch and body blocks
run in the same value environment as their parent, so they read outer Variables directly, and
autograd records whatever actually executed (gradients flow through the taken branch and every
loop iteration).
"""
from __future__ import annotations

import torch

from ..framework import core as _core
from ..framework.core import Tensor, _wrap
from . import program as P


def _flat(tree):
    """-> (leaves, rebuild(leaves))"""
    if isinstance(tree, (list, tuple)):
        parts = [_flat(t) for t in tree]
        leaves = [l for lv, _ in parts for l in lv]

        def build(vals, _t=type(tree), _parts=parts):
            out, k = [], 0
            for lv, b in _parts:
                out.append(b(vals[k:k + len(lv)]))
                k += len(lv)
            return _t(out)
        return leaves, build
    if isinstance(tree, dict):
        keys = list(tree)
        parts = [_flat(tree[k]) for k in keys]
        leaves = [l for lv, _ in parts for l in lv]

        def build(vals, _parts=parts):
            out, k = {}, 0
            for key, (lv, b) in zip(keys, _parts):
                out[key] = b(vals[k:k + len(lv)])
                k += len(lv)
            return out
        return leaves, build
    return [tree], lambda vals: vals[0]


def _produced(block):
    ids = set()
    for op in block.ops:
        ids.update(id(v) for v in P._iter_vars(op.outputs))
        ids.update(id(v) for v in P._iter_vars([p for p in op.attrs.get("placeholders", []) if p is not None]))
    return ids


def _captured(blocks, exclude=()):
    """outer Variables read by the ops of ``blocks`` (for pruning / serialisation)"""
    produced = set(id(v) for v in exclude)
    for b in blocks:
        produced |= _produced(b)
    seen, out = set(), []
    for b in blocks:
        for op in b.ops:
            srcs = list(P._iter_vars((op.args, op.kwargs)))
            if op.exec is not None:
                srcs += list(P._iter_vars(op.attrs.get("captured", [])))
            for v in srcs:
                if id(v) not in produced and id(v) not in seen:
                    seen.add(id(v))
                    out.append(v)
    return out


def _meta_var(block, like, name=None):
    t = like._t if isinstance(like, Tensor) else torch.as_tensor(like)
    v = P.Variable(block, t.to("meta") if t.device.type != "meta" else t, name)
    if isinstance(like, P.Variable) and like.declared_shape is not None:
        v.declared_shape = list(like.declared_shape)
    block.vars[v.name] = v
    return v


def _trace_branch(prog, fn, args=()):
    blk = prog._create_block()
    try:
        out = fn(*args) if fn is not None else None
    finally:
        prog._rollback()
    return blk, out


def _is_var(x):
    return isinstance(x, P.Variable)


def cond(pred, true_fn=None, false_fn=None, undefined=None):
    prog = P.default_main_program()
    parent = prog.current_block()
    tb, t_out = _trace_branch(prog, true_fn)
    fb, f_out = _trace_branch(prog, false_fn)
    t_leaves, build = _flat(t_out)
    f_leaves, _ = _flat(f_out)
    if len(t_leaves) != len(f_leaves):
        raise ValueError(f"cond: true_fn returns {len(t_leaves)} values, false_fn {len(f_leaves)}; both branches "
                         "must return the same structure")
    if undefined is not None:
        for leaves, other in ((t_leaves, f_leaves), (f_leaves, t_leaves)):
            for k, (a, b) in enumerate(zip(leaves, other)):
                if a is undefined and isinstance(b, Tensor):
                    leaves[k] = _wrap(torch.zeros(tuple(b._t.shape), dtype=b._t.dtype, device=_core.default_device()))
    outs = []
    for a, b in zip(t_leaves, f_leaves):
        if undefined is not None and a is undefined and b is undefined:
            outs.append(undefined)
            continue
        if isinstance(a, Tensor) or isinstance(b, Tensor):
            like = a if isinstance(a, Tensor) else b
            outs.append(_meta_var(parent, like))
        elif isinstance(a, (bool, int, float)) and isinstance(b, (bool, int, float)) and a != b:
            # Python scalars that depend on the branch (dy2static flags, counters) become tensors
            like = _wrap(torch.as_tensor(a if not isinstance(b, float) else b))
            outs.append(_meta_var(parent, like))
        else:
            if a != b:
                raise ValueError(f"cond: non-tensor outputs differ between branches ({a!r} vs {b!r})")
            outs.append(a)
    captured = _captured([tb, fb]) + [v for v in t_leaves + f_leaves if _is_var(v)]
    op = P.OpDesc("conditional_block", None, (), {"pred": pred}, outs,
                  attrs={"true_block": tb.idx, "false_block": fb.idx, "true_outs": t_leaves, "false_outs": f_leaves,
                         "captured": captured}, exec=_exec_cond)
    for v in outs:
        if _is_var(v):
            v.op = op
    parent.append_op(op)
    return build(outs)


def _truth(x):
    if isinstance(x, Tensor):
        return bool(x._t.reshape(-1)[0].item())
    return bool(x)


def _exec_cond(program, env, op):
    take = _truth(P._subst(op.kwargs["pred"], env))
    blk = program.blocks[op.attrs["true_block" if take else "false_block"]]
    P.run_block(program, blk, env)
    vals = P._subst(op.attrs["true_outs" if take else "false_outs"], env)
    for o, v in zip(op.outputs, vals):
        if _is_var(o):
            env[id(o)] = v if isinstance(v, Tensor) else _wrap(torch.as_tensor(v))


def while_loop(cond_fn, body_fn, loop_vars, undefined=None):
    """``undefined``: sentinel of loop variables not bound before the loop (dy2static); their
    placeholder stays that sentinel and their output takes the body's value"""
    prog = P.default_main_program()
    parent = prog.current_block()
    loop_vars = list(loop_vars)
    init = []
    for v in loop_vars:
        if isinstance(v, Tensor) or (undefined is not None and v is undefined):
            init.append(v)
        else:   # Python scalar loop variables become scalar tensors (their updates must be recorded)
            with _dynamic():
                init.append(_wrap(torch.as_tensor(v, device=_core.default_device())))
    is_undef = [undefined is not None and v is undefined for v in init]
    cb = prog._create_block()
    try:
        ph = [v if u else _meta_var(cb, v) for v, u in zip(init, is_undef)]
        c_out = cond_fn(*ph)
    finally:
        prog._rollback()
    bb = prog._create_block()
    try:
        b_out = body_fn(*ph)
    finally:
        prog._rollback()
    b_out = list(b_out) if isinstance(b_out, (list, tuple)) else [b_out]
    if len(b_out) != len(ph):
        raise ValueError(f"while_loop: body returns {len(b_out)} values for {len(ph)} loop variables")
    outs = []
    for v, u, b in zip(init, is_undef, b_out):
        if not u:
            outs.append(_meta_var(parent, v))
        elif isinstance(b, Tensor):
            outs.append(_meta_var(parent, b))
        else:
            raise ValueError("while_loop: a loop variable first bound in the body must be a tensor")
    ph = [p if not u else None for p, u in zip(ph, is_undef)]
    ph_ids = {id(v) for v in ph if v is not None}
    captured = _captured([cb, bb], exclude=[p for p in ph if p is not None]) + \
        [v for v in b_out if _is_var(v) and id(v) not in ph_ids]
    op = P.OpDesc("while", None, (), {"loop_vars": init}, outs,
                  attrs={"cond_block": cb.idx, "body_block": bb.idx, "placeholders": ph, "cond_out": c_out,
                         "body_outs": b_out, "captured": captured}, exec=_exec_while)
    for v in outs:
        v.op = op
    parent.append_op(op)
    return outs


def _exec_while(program, env, op):
    vals = P._subst(op.kwargs["loop_vars"], env)
    ph = op.attrs["placeholders"]
    cblk, bblk = program.blocks[op.attrs["cond_block"]], program.blocks[op.attrs["body_block"]]
    while True:
        for p, v in zip(ph, vals):
            if p is not None:
                env[id(p)] = v
        P.run_block(program, cblk, env)
        if not _truth(P._subst(op.attrs["cond_out"], env)):
            break
        P.run_block(program, bblk, env)
        vals = [v if isinstance(v, Tensor) else _wrap(torch.as_tensor(v)) for v in P._subst(op.attrs["body_outs"], env)]
    for o, v in zip(op.outputs, vals):
        if isinstance(v, Tensor):
            env[id(o)] = v


class _dynamic:
    def __enter__(self):
        self.prev = _core._mode.static
        _core._mode.static = False

    def __exit__(self, *a):
        _core._mode.static = self.prev
