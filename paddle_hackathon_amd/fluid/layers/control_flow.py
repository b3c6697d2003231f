"""``fluid.layers`` control flow (reference: python/paddle/fluid/layers/control_flow.py; executors
paddle/fluid/operators/controlflow/{while_op,conditional_block_op}.cc, recurrent_op.cc,
tensor_array_read_write_op.cc).

The block-structured builders — ``While``, ``Switch``, ``IfElse``, ``StaticRNN``,
``DynamicRNN`` — record their bodies into sub-blocks of the current Program and append ONE op
whose executor interprets the sub-block (repeatedly, per branch, or per time step) in the
enclosing value environment. Body ops that update an outer variable (``increment(i)``,
``less_than(..., cond=c)``, ``assign(x, output=y)``, ``array_write(..., array=a)``) append an
op whose output *is* that outer Variable, so later readers — including the next iteration —
see the new value. Tensor arrays are Python lists in the value environment.

``IfElse`` also runs eagerly in dygraph mode; the others are static-graph builders like the
reference's (dygraph code uses Python control flow or ``paddle.jit.to_static``).
"""
from __future__ import annotations

import torch

from ...framework.core import Tensor
from ...static import nn as SN
from ...static import program as P
from ._common import T, W, dev, write_to, is_static_var, static_mode, to_padded
from .. import core as fcore

__all__ = ["While", "Switch", "increment", "array_write", "create_array", "less_than", "less_equal", "greater_than",
           "greater_equal", "equal", "not_equal", "array_read", "array_length", "cond", "IfElse", "DynamicRNN",
           "StaticRNN", "reorder_lod_tensor_by_rank", "Print", "Assert", "is_empty", "case", "switch_case",
           "while_loop"]


def _truth(v):
    if isinstance(v, Tensor):
        return bool(v._t.reshape(-1)[0].item())
    return bool(v)


def _meta_like(block, like, name=None, shape=None):
    t = like._t if isinstance(like, Tensor) else torch.as_tensor(like)
    if shape is not None:
        t = torch.empty(shape, dtype=t.dtype, device="meta")
    v = P.Variable(block, t.to("meta") if t.device.type != "meta" else t, name)
    block.vars[v.name] = v
    return v


class _SubBlock:
    """records ops into a fresh sub-block of the current Program while active"""

    def __init__(self, on_exit=None):
        self.on_exit = on_exit

    def __enter__(self):
        self.prog = P.default_main_program()
        self.blk = self.prog._create_block()
        return self.blk

    def __exit__(self, et, *a):
        self.prog._rollback()
        if et is None and self.on_exit is not None:
            self.on_exit(self.blk)
        return False


def _require_static(what):
    if not static_mode():
        raise RuntimeError(f"fluid.layers.{what} builds a static Program: call paddle.enable_static() first "
                           "(dygraph code uses Python control flow or paddle.jit.to_static)")


def _captured(blocks, exclude=()):
    from ...static.control_flow import _captured as cap
    return cap(blocks, exclude)


# ----------------------------------------------------------------------------- comparisons / counters
def _cmp(fn, opname):
    def compute(x, y):
        return W(fn(T(x), T(y) if isinstance(y, Tensor) else y))

    def op(x, y, force_cpu=None, cond=None, name=None):
        r = _record_or_run(compute, opname, (x, y))
        return write_to(cond, r) if cond is not None else r
    op.__name__ = opname
    return op


less_than = _cmp(torch.lt, "less_than")
less_equal = _cmp(torch.le, "less_equal")
greater_than = _cmp(torch.gt, "greater_than")
greater_equal = _cmp(torch.ge, "greater_equal")
equal = _cmp(torch.eq, "equal")
not_equal = _cmp(torch.ne, "not_equal")


def _increment(x, value):
    return W(T(x) + value)


def increment(x, value=1.0, in_place=True):
    r = _record_or_run(_increment, "increment", (x, value))
    if in_place:
        return write_to(x, r)
    return r


def _record_or_run(fn, name, args):
    from ...framework.dispatch import static_op
    return static_op(fn, name)(*args)


def is_empty(x, cond=None):
    r = _record_or_run(lambda v: W(torch.tensor([T(v).numel() == 0], device=dev())), "is_empty", (x,))
    return write_to(cond, r) if cond is not None else r


# ----------------------------------------------------------------------------- tensor arrays
class _ArrayVar(P.Variable):
    """static-mode LoDTensorArray: its value in the executor environment is a Python list"""

    def __init__(self, block, dtype, name=None):
        super().__init__(block, torch.empty([0], dtype=dtype, device="meta"), name or P._core._unique_name("array"))
        self.elem_meta = None
        block.vars[self.name] = self


def create_array(dtype, initialized_list=None):
    if static_mode():
        blk = P.default_main_program().current_block()
        arr = _ArrayVar(blk, fcore.convert_dtype(dtype))
        init = list(initialized_list or [])
        if init:
            arr.elem_meta = init[0]
        op = P.OpDesc("create_array", lambda *xs: list(xs), tuple(init), {}, arr)
        blk.append_op(op)
        return arr
    return fcore.LoDTensorArray(initialized_list or [])


def _array_write(arr, x, i):
    out = list(arr or [])
    k = int(T(i).reshape(-1)[0].item()) if isinstance(i, Tensor) else int(i)
    while len(out) <= k:
        out.append(None)
    out[k] = x
    return out


def array_write(x, i, array=None):
    if static_mode() and (is_static_var(x) or isinstance(array, _ArrayVar)):
        blk = P.default_main_program().current_block()
        if array is None:
            array = create_array(x.dtype)
        array.elem_meta = x
        op = P.OpDesc("write_to_array", _array_write, (array, x, i), {}, array)
        blk.append_op(op)
        return array
    if array is None:
        array = fcore.LoDTensorArray()
    new = _array_write(array, x, i)
    array[:] = new
    return array


def _array_read(arr, i):
    k = int(T(i).reshape(-1)[0].item()) if isinstance(i, Tensor) else int(i)
    return arr[k]


def array_read(array, i):
    if isinstance(array, _ArrayVar):
        blk = P.default_main_program().current_block()
        if array.elem_meta is None:
            raise ValueError("array_read: nothing was written to this array before the read was recorded")
        out = _meta_like(blk, array.elem_meta)
        op = P.OpDesc("read_from_array", _array_read, (array, i), {}, out)
        out.op = op
        blk.append_op(op)
        return out
    return _array_read(array, i)


def array_length(array):
    if isinstance(array, _ArrayVar):
        blk = P.default_main_program().current_block()
        out = _meta_like(blk, torch.zeros(1, dtype=torch.long))
        op = P.OpDesc("lod_array_length", lambda a: W(torch.tensor([len(a)], dtype=torch.long, device=dev())),
                      (array,), {}, out)
        out.op = op
        blk.append_op(op)
        return out
    return W(torch.tensor([len(array)], dtype=torch.long, device=dev()))


# ----------------------------------------------------------------------------- While
class While:
    """``with While(cond).block(): ...`` — runs the body while ``cond`` (a bool [1] Variable the
    body updates) is true"""

    def __init__(self, cond, is_test=False, name=None):
        self.cond_var = cond
        self.is_test = is_test

    def block(self):
        _require_static("While")
        return _SubBlock(self._finish)

    def _finish(self, body):
        prog = P.default_main_program()
        parent = prog.current_block()
        written = _outer_writes(body)
        op = P.OpDesc("while", None, (), {"Condition": self.cond_var}, written,
                      attrs={"sub_block": body.idx, "captured": _captured([body]) + [self.cond_var],
                             "is_test": self.is_test}, exec=_exec_while)
        parent.append_op(op)


def _outer_writes(blk):
    outs, seen = [], set()
    for op in blk.ops:
        if op.attrs.get("inplace_write") or op.type in ("write_to_array",):
            for v in P._iter_vars(op.outputs):
                if v.block is not blk and id(v) not in seen:
                    seen.add(id(v))
                    outs.append(v)
    return outs


def _exec_while(program, env, op):
    body = program.blocks[op.attrs["sub_block"]]
    c = op.kwargs["Condition"]
    n = 0
    while _truth(env[id(c)]):
        P.run_block(program, body, env)
        n += 1
        if n > 10_000_000:
            raise RuntimeError("While: more than 1e7 iterations")


# ----------------------------------------------------------------------------- Switch
class Switch:
    """``with Switch() as s: with s.case(c1): ... with s.default(): ...`` — the first case whose
    condition holds runs (conditional_block chain)"""

    def __init__(self, name=None):
        self.cases = []
        self.default_blk = None
        self.inside = False

    def __enter__(self):
        _require_static("Switch")
        self.inside = True
        return self

    def case(self, condition):
        if not self.inside:
            raise ValueError("Switch.case must be used inside `with Switch()`")
        return _SubBlock(lambda b: self.cases.append((condition, b)))

    def default(self):
        if not self.inside:
            raise ValueError("Switch.default must be used inside `with Switch()`")

        def done(b):
            self.default_blk = b
        return _SubBlock(done)

    def __exit__(self, et, *a):
        self.inside = False
        if et is not None:
            return False
        blocks = [b for _, b in self.cases] + ([self.default_blk] if self.default_blk else [])
        written = []
        for b in blocks:
            written += [v for v in _outer_writes(b) if all(v is not w for w in written)]
        op = P.OpDesc("switch", None, (), {"conds": [c for c, _ in self.cases]}, written,
                      attrs={"case_blocks": [b.idx for _, b in self.cases],
                             "default_block": self.default_blk.idx if self.default_blk else -1,
                             "captured": _captured(blocks) + [c for c, _ in self.cases]}, exec=_exec_switch)
        P.default_main_program().current_block().append_op(op)
        return False


def _exec_switch(program, env, op):
    for c, bi in zip(op.kwargs["conds"], op.attrs["case_blocks"]):
        if _truth(P._subst(c, env)):
            P.run_block(program, program.blocks[bi], env)
            return
    if op.attrs["default_block"] >= 0:
        P.run_block(program, program.blocks[op.attrs["default_block"]], env)


# ----------------------------------------------------------------------------- IfElse
class IfElse:
    """row-wise if/else: ``cond`` is a bool [N, 1] tensor; inside ``true_block()`` the inputs are
    the rows where it holds, inside ``false_block()`` the others; ``ie()`` merges each output's
    rows back into batch order"""

    def __init__(self, cond, name=None):
        self.cond = cond
        self.branch = None
        self.static = is_static_var(cond) and static_mode()
        self.inputs = {True: [], False: []}      # (placeholder, outer var) in static mode
        self.outs = {True: [], False: []}
        self.blocks = {}

    def _guard(self, flag):
        ie = self

        class _G:
            def __enter__(self_):
                ie.branch = flag
                if ie.static:
                    self_.sb = _SubBlock(lambda b: ie.blocks.__setitem__(flag, b))
                    self_.sb.__enter__()
                return ie

            def __exit__(self_, et, *a):
                if ie.static:
                    self_.sb.__exit__(et, *a)
                ie.branch = None
                return False
        return _G()

    def true_block(self):
        return self._guard(True)

    def false_block(self):
        return self._guard(False)

    def _mask(self):
        return T(self.cond).reshape(-1).bool()

    def input(self, x):
        if self.branch is None:
            raise ValueError("IfElse.input must be called inside true_block() / false_block()")
        if self.static:
            ph = _meta_like(P.default_main_program().current_block(), x)
            self.inputs[self.branch].append((ph, x))
            return ph
        m = self._mask() if self.branch else ~self._mask()
        return W(T(x)[m])

    def output(self, *outs):
        if self.branch is None:
            raise ValueError("IfElse.output must be called inside true_block() / false_block()")
        self.outs[self.branch].extend(outs)

    def __call__(self):
        t_out, f_out = self.outs[True], self.outs[False]
        if t_out and f_out and len(t_out) != len(f_out):
            raise ValueError("IfElse: both branches must produce the same number of outputs")
        if not self.static:
            m = self._mask()
            res = []
            for a, b in zip(t_out or [None] * len(f_out), f_out or [None] * len(t_out)):
                like = T(a if a is not None else b)
                out = like.new_zeros([m.shape[0]] + list(like.shape[1:]))
                if a is not None:
                    out = out.index_put((m.nonzero().reshape(-1),), T(a))
                if b is not None:
                    out = out.index_put(((~m).nonzero().reshape(-1),), T(b))
                res.append(W(out))
            return res
        parent = P.default_main_program().current_block()
        n = len(t_out or f_out)
        outs = [_meta_like(parent, (t_out or f_out)[k]) for k in range(n)]
        blocks = [b for b in (self.blocks.get(True), self.blocks.get(False)) if b is not None]
        phs = [p for p, _ in self.inputs[True] + self.inputs[False]]
        op = P.OpDesc("ifelse", None, (), {"cond": self.cond,
                                           "inputs": [x for _, x in self.inputs[True] + self.inputs[False]]}, outs,
                      attrs={"true_block": self.blocks[True].idx if True in self.blocks else -1,
                             "false_block": self.blocks[False].idx if False in self.blocks else -1,
                             "true_inputs": self.inputs[True], "false_inputs": self.inputs[False],
                             "true_outs": t_out, "false_outs": f_out,
                             "captured": _captured(blocks, exclude=phs)}, exec=_exec_ifelse)
        for v in outs:
            v.op = op
        parent.append_op(op)
        return outs


def _exec_ifelse(program, env, op):
    m = T(P._subst(op.kwargs["cond"], env)).reshape(-1).bool()
    parts = {}
    for flag, key in ((True, "true"), (False, "false")):
        bi = op.attrs[f"{key}_block"]
        idx = (m if flag else ~m).nonzero().reshape(-1)
        for ph, x in op.attrs[f"{key}_inputs"]:
            env[id(ph)] = W(T(P._subst(x, env))[idx])
        if bi >= 0:
            P.run_block(program, program.blocks[bi], env)
        parts[flag] = (idx, [P._subst(o, env) for o in op.attrs[f"{key}_outs"]])
    for k, o in enumerate(op.outputs):
        like = None
        for flag in (True, False):
            if len(parts[flag][1]) > k:
                like = T(parts[flag][1][k])
        out = like.new_zeros([m.shape[0]] + list(like.shape[1:]))
        for flag in (True, False):
            idx, vals = parts[flag]
            if len(vals) > k:
                out = out.index_put((idx,), T(vals[k]))
        env[id(o)] = W(out)


# ----------------------------------------------------------------------------- StaticRNN
class StaticRNN:
    """fixed-length recurrence over dim 0 of its step inputs ([T, B, ...]) (recurrent_op.cc)"""

    def __init__(self, name=None):
        self.step_inputs = []        # (placeholder, outer var)
        self.memories = []           # dict(ph, init, shape, value, ref, ref_idx, init_idx, update)
        self.step_outputs = []
        self.block_idx = None
        self.outputs = None
        self._inside = False

    def step(self):
        _require_static("StaticRNN")
        rnn = self

        class _G(_SubBlock):
            def __enter__(self_):
                rnn._inside = True
                return super().__enter__()

            def __exit__(self_, et, *a):
                rnn._inside = False
                return super().__exit__(et, *a)
        return _G(self._finish)

    def step_input(self, x):
        blk = P.default_main_program().current_block()
        ph = _meta_like(blk, x, shape=list(x._t.shape[1:]))
        self.step_inputs.append((ph, x))
        return ph

    def memory(self, init=None, shape=None, batch_ref=None, init_value=0.0, init_batch_dim_idx=0,
               ref_batch_dim_idx=1):
        blk = P.default_main_program().current_block()
        if init is not None:
            ph = _meta_like(blk, init)
        else:
            shp = [1 if s == -1 else s for s in shape]
            ph = _meta_like(blk, torch.zeros(shp))
        self.memories.append({"ph": ph, "init": init, "shape": shape, "value": init_value, "ref": batch_ref,
                              "ref_idx": ref_batch_dim_idx, "init_idx": init_batch_dim_idx, "update": None})
        return ph

    def update_memory(self, mem, var):
        for m in self.memories:
            if m["ph"] is mem:
                m["update"] = var
                return
        raise ValueError("update_memory: unknown memory")

    def step_output(self, o):
        self.step_outputs.append(o)

    def output(self, *outputs):
        for o in outputs:
            self.step_output(o)

    def _finish(self, body):
        parent = P.default_main_program().current_block()
        steps = self.step_inputs[0][1]._t.shape[0] if self.step_inputs else 1
        outs = [_meta_like(parent, o, shape=[steps] + list(o._t.shape)) for o in self.step_outputs]
        phs = [p for p, _ in self.step_inputs] + [m["ph"] for m in self.memories]
        op = P.OpDesc("recurrent", None, (), {"inputs": [x for _, x in self.step_inputs],
                                              "inits": [m["init"] for m in self.memories if m["init"] is not None]},
                      outs, attrs={"sub_block": body.idx, "step_inputs": self.step_inputs, "memories": self.memories,
                                   "step_outputs": self.step_outputs,
                                   "captured": _captured([body], exclude=phs)}, exec=_exec_static_rnn)
        for v in outs:
            v.op = op
        parent.append_op(op)
        self.outputs = outs

    def __call__(self, *args, **kwargs):
        if self.outputs is None:
            raise ValueError("StaticRNN: call rnn() after the `with rnn.step()` block")
        return self.outputs[0] if len(self.outputs) == 1 else self.outputs


def _batch_of(ref, ref_idx, step_inputs, env):
    for ph, x in step_inputs:
        if ref is ph:
            return T(P._subst(x, env)).shape[1]
    return T(P._subst(ref, env)).shape[ref_idx]


def _exec_static_rnn(program, env, op):
    body = program.blocks[op.attrs["sub_block"]]
    xs = [(ph, T(P._subst(x, env))) for ph, x in op.attrs["step_inputs"]]
    steps = xs[0][1].shape[0] if xs else 1
    mems = []
    for m in op.attrs["memories"]:
        if m["init"] is not None:
            mems.append(P._subst(m["init"], env))
        else:
            b = _batch_of(m["ref"], m["ref_idx"], op.attrs["step_inputs"], env)
            shp = [b if s == -1 else s for s in m["shape"]]
            mems.append(W(torch.full(shp, float(m["value"]), device=dev())))
    collected = [[] for _ in op.outputs]
    for t in range(steps):
        for ph, x in xs:
            env[id(ph)] = W(x[t])
        for m, v in zip(op.attrs["memories"], mems):
            env[id(m["ph"])] = v
        P.run_block(program, body, env)
        for k, o in enumerate(op.attrs["step_outputs"]):
            collected[k].append(T(P._subst(o, env)))
        mems = [P._subst(m["update"], env) if m["update"] is not None else v
                for m, v in zip(op.attrs["memories"], mems)]
    for o, parts in zip(op.outputs, collected):
        env[id(o)] = W(torch.stack(parts, 0))


# ----------------------------------------------------------------------------- DynamicRNN
class DynamicRNN:
    """recurrence over variable-length (LoD) sequences: step t runs on the sequences longer than
    t, sorted by length (the lod_rank_table / shrink_memory scheme of the reference)"""

    def __init__(self, name=None):
        self.step_inputs, self.static_inputs, self.memories, self.outs = [], [], [], []
        self.outputs = None

    def block(self):
        _require_static("DynamicRNN")
        return _SubBlock(self._finish)

    def step_input(self, x, level=0):
        ph = _meta_like(P.default_main_program().current_block(), x, shape=[1] + list(x._t.shape[1:]))
        self.step_inputs.append((ph, x))
        return ph

    def static_input(self, x):
        ph = _meta_like(P.default_main_program().current_block(), x)
        self.static_inputs.append((ph, x))
        return ph

    def memory(self, init=None, shape=None, value=0.0, need_reorder=False, dtype="float32"):
        blk = P.default_main_program().current_block()
        ph = _meta_like(blk, init) if init is not None else \
            _meta_like(blk, torch.zeros([1] + list(shape), dtype=fcore.convert_dtype(dtype)))
        self.memories.append({"ph": ph, "init": init, "shape": shape, "value": value, "reorder": need_reorder,
                              "dtype": dtype, "update": None})
        return ph

    def update_memory(self, ex_mem, new_mem):
        for m in self.memories:
            if m["ph"] is ex_mem:
                m["update"] = new_mem
                return
        raise ValueError("update_memory: unknown memory")

    def output(self, *outputs):
        self.outs.extend(outputs)

    def _finish(self, body):
        parent = P.default_main_program().current_block()
        outs = [_meta_like(parent, o) for o in self.outs]
        phs = [p for p, _ in self.step_inputs + self.static_inputs] + [m["ph"] for m in self.memories]
        op = P.OpDesc("dynamic_rnn", None, (), {"inputs": [x for _, x in self.step_inputs + self.static_inputs],
                                                "inits": [m["init"] for m in self.memories if m["init"] is not None]},
                      outs, attrs={"sub_block": body.idx, "step_inputs": self.step_inputs,
                                   "static_inputs": self.static_inputs, "memories": self.memories,
                                   "step_outputs": self.outs, "captured": _captured([body], exclude=phs)},
                      exec=_exec_dynamic_rnn)
        for v in outs:
            v.op = op
        parent.append_op(op)
        self.outputs = outs

    def __call__(self, *args, **kwargs):
        if self.outputs is None:
            raise ValueError("DynamicRNN: call drnn() after the `with drnn.block()` block")
        return self.outputs[0] if len(self.outputs) == 1 else self.outputs


def _exec_dynamic_rnn(program, env, op):
    body = program.blocks[op.attrs["sub_block"]]
    first = P._subst(op.attrs["step_inputs"][0][1], env)
    off = fcore.lod_of(first)[-1] if fcore.lod_of(first) else list(range(T(first).shape[0] + 1))
    lens = fcore._lengths_from_offsets(off)
    order = sorted(range(len(lens)), key=lambda i: -lens[i])     # stable: ties keep input order
    xs = [(ph, T(P._subst(x, env))) for ph, x in op.attrs["step_inputs"]]
    statics = [(ph, T(P._subst(x, env))[torch.tensor(order, device=dev())]) for ph, x in op.attrs["static_inputs"]]
    mems = []
    for m in op.attrs["memories"]:
        if m["init"] is not None:
            v = T(P._subst(m["init"], env))
            mems.append(v[torch.tensor(order, device=v.device)] if m["reorder"] else v)
        else:
            mems.append(torch.full([len(lens)] + list(m["shape"]), float(m["value"]), device=dev(),
                                   dtype=fcore.convert_dtype(m["dtype"])))
    rows = [[[] for _ in lens] for _ in op.outputs]
    for t in range(max(lens) if lens else 0):
        active = [s for s in order if lens[s] > t]
        n = len(active)
        for ph, x in xs:
            env[id(ph)] = W(x[torch.tensor([off[s] + t for s in active], device=x.device)])
        for ph, x in statics:
            env[id(ph)] = W(x[:n])
        for m, v in zip(op.attrs["memories"], mems):
            env[id(m["ph"])] = W(v[:n])
        P.run_block(program, body, env)
        for k, o in enumerate(op.attrs["step_outputs"]):
            val = T(P._subst(o, env))
            for j, s in enumerate(active):
                rows[k][s].append(val[j])
        new = []
        for m, v in zip(op.attrs["memories"], mems):
            if m["update"] is None:
                new.append(v)
                continue
            u = T(P._subst(m["update"], env))
            new.append(torch.cat([u, v[n:]], 0) if n < v.shape[0] else u)
        mems = new
    for o, per_seq in zip(op.outputs, rows):
        flat = torch.stack([r for seq in per_seq for r in seq], 0)
        out = W(flat)
        out._lod = [list(off)]
        env[id(o)] = out


# ----------------------------------------------------------------------------- rank table
class _RankTable:
    def __init__(self, items):
        self.items = items            # [(index, length)] sorted by length desc


def lod_rank_table(x, level=0):
    off = fcore.lod_of(x)[level]
    lens = fcore._lengths_from_offsets(off)
    return _RankTable(sorted(((i, n) for i, n in enumerate(lens)), key=lambda p: -p[1]))


def reorder_lod_tensor_by_rank(x, rank_table):
    """reorder the sequences of ``x`` (or its rows, without LoD) in the rank table's order"""
    t = T(x)
    order = [i for i, _ in rank_table.items]
    lod = fcore.lod_of(x)
    if not lod:
        return W(t[torch.tensor(order, device=t.device)])
    off = lod[0]
    parts = [t[off[i]:off[i + 1]] for i in order]
    out = W(torch.cat(parts, 0))
    out._lod = [fcore._offsets_from_lengths([off[i + 1] - off[i] for i in order])]
    return out


# ----------------------------------------------------------------------------- functional control flow
def cond(pred, true_fn=None, false_fn=None, name=None):
    return SN.cond(pred, true_fn, false_fn, name)


def case(pred_fn_pairs, default=None, name=None):
    return SN.case(pred_fn_pairs, default, name)


def switch_case(branch_index, branch_fns, default=None, name=None):
    return SN.switch_case(branch_index, branch_fns, default, name)


def while_loop(cond, body, loop_vars, is_test=False, name=None):
    return SN.while_loop(cond, body, loop_vars, is_test, name)


class _Printer:
    """the reference print op (print_op.cc): at most ``first_n`` prints (-1: every run) of the
    tensor's name, dtype, shape, LoD and its first ``summarize`` values (-1: all), prefixed by
    ``message``; returns its input unchanged. Forward phase only (print_phase "backward" prints
    nothing: gradients have no print op here)."""

    def __init__(self, name, first_n, message, summarize, show_name, show_type, show_shape, show_lod, phase):
        self.name, self.first_n, self.message, self.summarize = name, first_n, message, summarize
        self.flags = (show_name, show_type, show_shape, show_lod)
        self.phase, self.count = phase, 0

    def __call__(self, x):
        if self.phase == "backward" or (0 <= self.first_n <= self.count):
            return x
        self.count += 1
        t = T(x)
        flat = t.detach().reshape(-1)
        vals = flat[:self.summarize] if self.summarize >= 0 else flat
        lines = [self.message] if self.message else []
        if self.flags[0] and self.name:
            lines.append(f"Variable: {self.name}")
        if self.flags[3]:
            lines.append(f"  - lod: {fcore.lod_of(x) or '{}'}")
        if self.flags[2]:
            lines.append(f"  - shape: {list(t.shape)}")
        if self.flags[1]:
            lines.append(f"  - dtype: {str(t.dtype).replace('torch.', '')}")
        lines.append(f"  - data: {vals.cpu().tolist()}")
        print("\n".join(lines), flush=True)
        return x


def Print(input, first_n=-1, message=None, summarize=20, print_tensor_name=True, print_tensor_type=True,
          print_tensor_shape=True, print_tensor_lod=True, print_phase="both"):
    """control_flow.py:Print — records one ``print`` op (nothing is printed while the Program is
    built; static/program.py registers its InferMeta as the identity)"""
    pr = _Printer(getattr(input, "name", None), first_n, message, summarize, print_tensor_name, print_tensor_type,
                  print_tensor_shape, print_tensor_lod, print_phase)

    def print_(x):
        return pr(x)
    out = _record_or_run(print_, "print", (input,))
    from ...static.program import set_ref_op
    set_ref_op(out, "print", {"In": [input]}, {"Out": [out]}, {
        "first_n": int(first_n), "message": message or "", "summarize": int(summarize),
        "print_tensor_name": bool(print_tensor_name), "print_tensor_type": bool(print_tensor_type),
        "print_tensor_shape": bool(print_tensor_shape), "print_tensor_lod": bool(print_tensor_lod),
        "print_phase": str(print_phase).upper(), "is_forward": True})
    return out


def _assert(c, data, summarize):
    if not _truth(c):
        shown = [T(d).reshape(-1)[:summarize].tolist() for d in (data or [])]
        raise ValueError(f"Assert failed: condition is False; data: {shown}")
    return c


def Assert(cond, data=None, summarize=20, name=None):
    return _record_or_run(_assert, "assert", (cond, list(data) if data else None, summarize))


_ = to_padded
