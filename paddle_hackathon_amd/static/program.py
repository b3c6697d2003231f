"""Static graph: Program / Block / Variable, recording and the replay Executor
(reference: python/paddle/fluid/framework.py, executor.py, backward.py, compiler.py;
paddle/fluid/framework/{program_desc,block_desc,op_desc,executor,new_executor/*}).

Recording: in static mode every public op call whose arguments contain a ``Variable``
appends an ``OpDesc`` (op type = qualified op name, bound arguments, output Variables)
to the current block; output shapes/dtypes come from running the op on ``meta``
tensors (our InferMeta). Parameters are real device tensors living in the global scope.

Execution: ``Executor.run`` interprets the op list against a value environment —
feeds bound to data Variables, parameters by reference — so autograd, the HIP kernels
and the fused optimizers run exactly as in dynamic mode. ``CompiledProgram`` can freeze
a forward-only program into a HIP graph (torch.cuda.CUDAGraph on ROCm) replayed per run.

Serialisation: programs are lists of registered op names + JSON-able argument trees, so a
program round-trips through ``serialize_program`` / ``save_inference_model``.
"""
from __future__ import annotations

import collections
import contextlib
import copy
import inspect
import itertools
import json
import os
import threading
import time
import weakref

import numpy as np
import torch

from ..framework import core as _core
from ..framework.core import Tensor, Parameter, _wrap, convert_dtype, dtype_to_str

__all__ = ["Variable", "Program", "Block", "OpDesc", "record_op", "set_ref_op", "default_main_program", "default_startup_program",
           "program_guard", "data", "Executor", "global_scope", "scope_guard", "append_backward", "gradients",
           "minimize_static", "enable_static", "disable_static", "name_scope", "OP_REGISTRY", "CompiledProgram",
           "BuildStrategy", "ExecutionStrategy", "InputSpec", "Scope"]

OP_REGISTRY = {}
_var_ids = itertools.count()


class InputSpec:
    """Shape/dtype/name of a program input (reference: python/paddle/static/input.py)."""

    def __init__(self, shape, dtype="float32", name=None, stop_gradient=False):
        self.shape = [(-1 if s is None else int(s)) for s in shape]
        self.dtype = convert_dtype(dtype)
        self.name = name
        self.stop_gradient = stop_gradient

    @classmethod
    def from_tensor(cls, tensor, name=None):
        return cls(tensor.shape, tensor.dtype, name or tensor.name)

    @classmethod
    def from_numpy(cls, ndarray, name=None):
        return cls(ndarray.shape, ndarray.dtype, name)

    def batch(self, batch_size):
        return InputSpec([batch_size] + self.shape, self.dtype, self.name)

    def unbatch(self):
        return InputSpec(self.shape[1:], self.dtype, self.name)

    def __repr__(self):
        return f"InputSpec(shape={self.shape}, dtype={self.dtype}, name={self.name})"

    def __eq__(self, other):
        return isinstance(other, InputSpec) and (self.shape, self.dtype, self.name) == (other.shape, other.dtype, other.name)

    def __hash__(self):
        return hash((tuple(self.shape), self.dtype, self.name))


class Variable(Tensor):
    """A symbolic tensor of a static Program. ``_t`` is a meta tensor (shape/dtype only)."""

    __slots__ = ()

    def __init__(self, block, meta, name=None, declared_shape=None, is_data=False, persistable=False, stop_gradient=True):
        self._t = meta
        self._name = name or f"_generated_var_{next(_var_ids)}"
        self._persistable = persistable
        self.block = block
        self.is_data = is_data
        self.declared_shape = declared_shape
        self.need_grad = not stop_gradient
        self.op = None

    @property
    def shape(self):
        if self.declared_shape is not None:
            return list(self.declared_shape)
        return list(self._t.shape) or [1]

    @property
    def stop_gradient(self):
        return not self.need_grad

    @stop_gradient.setter
    def stop_gradient(self, v):
        self.need_grad = not v

    def numpy(self):
        raise RuntimeError("a static Variable has no value; fetch it with Executor.run")

    def __repr__(self):
        return f"Variable(name={self.name}, shape={self.shape}, dtype={dtype_to_str(self._t.dtype)})"

    def __bool__(self):
        raise TypeError("a static Variable has no truth value; use paddle.static.nn.cond")

    def __len__(self):
        return self.shape[0]

    # augmented assignment on a symbolic tensor records an out-of-place op (an in-place update of
    # the meta tensor would vanish from the program)
    def __iadd__(self, o):
        return self + o

    def __isub__(self, o):
        return self - o

    def __imul__(self, o):
        return self * o

    def __itruediv__(self, o):
        return self / o

    def __deepcopy__(self, memo):
        return self

    def to_string(self, throw_on_error=False, with_details=False):
        return repr(self)


class OpDesc:
    """One recorded op: ``type`` (registered qualified op name, or a control-flow op type), the
    bound arguments (``kwargs``; Variables are the inputs, everything else the attributes) and the
    output Variables. Control-flow ops (``conditional_block``, ``while``) carry an ``exec`` handler
    that runs their sub-blocks (static/control_flow.py)."""
    __slots__ = ("type", "fn", "args", "kwargs", "outputs", "attrs", "exec")

    def __init__(self, type, fn, args, kwargs, outputs, attrs=None, exec=None):
        self.type, self.fn, self.args, self.kwargs, self.outputs = type, fn, args, kwargs, outputs
        self.attrs = attrs or {}
        self.exec = exec

    def input_arg_names(self):
        return [v.name for v in _iter_vars((self.args, self.kwargs))]

    def output_arg_names(self):
        return [v.name for v in _iter_vars(self.outputs)]

    def __repr__(self):
        return f"{{{', '.join(self.output_arg_names())}}} = {self.type}({', '.join(self.input_arg_names())})"


class Block:
    def __init__(self, program, idx=0, parent_idx=-1):
        self.program, self.idx, self.parent_idx = program, idx, parent_idx
        self.ops = []
        self.vars = {}

    def var(self, name):
        return self.vars[name]

    def has_var(self, name):
        return name in self.vars

    def all_parameters(self):
        return [v for v in self.vars.values() if isinstance(v, Parameter)]

    def append_op(self, op):
        if _OP_DEVICE[0] is not None and "op_device" not in op.attrs:   # static.device_guard
            op.attrs["op_device"] = _OP_DEVICE[0]
        self.ops.append(op)
        return op

    def create_var(self, name=None, shape=None, dtype="float32", persistable=False, **kw):
        meta = torch.empty([1 if s in (None, -1) else s for s in (shape or [])], dtype=convert_dtype(dtype), device="meta")
        v = Variable(self, meta, name, declared_shape=shape, persistable=persistable)
        self.vars[v.name] = v
        return v

    def __repr__(self):
        return "\n".join(repr(o) for o in self.ops)


class Program:
    _ids = itertools.count()

    def __init__(self):
        self.blocks = [Block(self)]
        self.random_seed = 0
        self._id = next(Program._ids)
        self._is_test = False
        self._hip_graph_cache = {}

    def global_block(self):
        return self.blocks[0]

    def block(self, i):
        return self.blocks[i]

    def current_block(self):
        return self.blocks[self._cur] if hasattr(self, "_cur") else self.blocks[0]

    def _create_block(self, parent_idx=None):
        """new sub-block (control flow) under the current one; recording goes there until
        _rollback()"""
        parent = self.current_block().idx if parent_idx is None else parent_idx
        b = Block(self, len(self.blocks), parent)
        self.blocks.append(b)
        self._stack = getattr(self, "_stack", []) + [getattr(self, "_cur", 0)]
        self._cur = b.idx
        return b

    def _rollback(self):
        self._cur = self._stack.pop() if getattr(self, "_stack", None) else 0

    @property
    def num_blocks(self):
        return len(self.blocks)

    def list_vars(self):
        return list(self.global_block().vars.values())

    def all_parameters(self):
        seen, out = set(), []
        for op in (o for b in self.blocks for o in b.ops):
            for a in _iter_tensors((op.args, op.kwargs, op.attrs.get("captured", []))):
                if isinstance(a, Parameter) and id(a) not in seen:
                    seen.add(id(a))
                    out.append(a)
        return out

    def clone(self, for_test=False):
        p = Program()
        p.random_seed = self.random_seed
        blk = p.global_block()
        blk.vars = dict(self.global_block().vars)
        for op in self.global_block().ops:
            if for_test and is_train_op(op):
                continue   # drop backward / optimizer ops
            kwargs = dict(op.kwargs)
            if for_test:
                for k in ("training", "is_test"):
                    if k in kwargs:
                        kwargs[k] = (k == "is_test")
                if "use_global_stats" in kwargs and "training" in op.kwargs:
                    pass
            blk.ops.append(OpDesc(op.type, op.fn, op.args, kwargs, op.outputs, dict(op.attrs), op.exec))
        p.blocks += self.blocks[1:]   # control-flow sub-blocks are shared (their ops reference them)
        p._is_test = for_test
        return p

    def __repr__(self):
        return f"Program(ops={len(self.global_block().ops)})\n" + repr(self.global_block())

    to_string = lambda self, throw_on_error=False, with_details=False: repr(self)  # noqa: E731

    def state_dict(self, mode="all", scope=None):
        return {p.name: p for p in self.all_parameters()}

    def set_state_dict(self, state_dict, scope=None):
        own = {p.name: p for p in self.all_parameters()}
        for k, v in state_dict.items():
            if k in own:
                own[k].set_value(v.numpy() if isinstance(v, Tensor) else np.asarray(v))

    def _prune(self, targets):
        p = self.clone()
        targets = targets if isinstance(targets, (list, tuple)) else [targets]
        p.global_block().ops = prune_ops(p.global_block().ops, [t for t in targets if isinstance(t, Variable)])
        return p


class _State:
    main = None
    startup = None


_state = _State()
_state.main = Program()
_state.startup = Program()


def default_main_program():
    return _state.main


def default_startup_program():
    return _state.startup


@contextlib.contextmanager
def program_guard(main_program, startup_program=None):
    old_main, old_startup = _state.main, _state.startup
    _state.main = main_program
    if startup_program is not None:
        _state.startup = startup_program
    try:
        yield
    finally:
        _state.main, _state.startup = old_main, old_startup


@contextlib.contextmanager
def name_scope(prefix=None):
    yield


def enable_static():
    _core._mode.static = True


def disable_static(place=None):
    _core._mode.static = False
    if place is not None:
        _core.set_device(place)


# ----------------------------------------------------------------------------- data
def data(name, shape, dtype=None, lod_level=0):
    dt = convert_dtype(dtype) or _core._default_dtype
    shape = [(-1 if s is None else int(s)) for s in shape]
    meta = torch.empty([1 if s == -1 else s for s in shape], dtype=dt, device="meta")
    blk = default_main_program().global_block()
    v = Variable(blk, meta, name, declared_shape=shape, is_data=True)
    v.lod_level = int(lod_level or 0)
    blk.vars[name] = v
    return v


# ----------------------------------------------------------------------------- recording
def _iter_vars(tree):
    if isinstance(tree, Variable):
        yield tree
    elif isinstance(tree, (list, tuple)):
        for t in tree:
            yield from _iter_vars(t)
    elif isinstance(tree, dict):
        for t in tree.values():
            yield from _iter_vars(t)


def _iter_tensors(tree):
    if isinstance(tree, Tensor):
        yield tree
    elif isinstance(tree, (list, tuple)):
        for t in tree:
            yield from _iter_tensors(t)
    elif isinstance(tree, dict):
        for t in tree.values():
            yield from _iter_tensors(t)


def _has_var(tree):
    return next(_iter_vars(tree), None) is not None


def _to_meta(tree):
    if isinstance(tree, Variable):
        return _wrap(tree._t)
    if isinstance(tree, Tensor):
        return _wrap(tree._t.to("meta"))
    if isinstance(tree, torch.Tensor):
        return tree.to("meta")
    if isinstance(tree, list):
        return [_to_meta(t) for t in tree]
    if isinstance(tree, tuple):
        return tuple(_to_meta(t) for t in tree)
    if isinstance(tree, dict):
        return {k: _to_meta(v) for k, v in tree.items()}
    return tree


def _outputs_to_vars(tree, block):
    if isinstance(tree, Tensor):
        v = Variable(block, tree._t if tree._t.device.type == "meta" else tree._t.to("meta"))
        block.vars[v.name] = v
        return v
    if isinstance(tree, list):
        return [_outputs_to_vars(t, block) for t in tree]
    if isinstance(tree, tuple):
        return tuple(_outputs_to_vars(t, block) for t in tree)
    return tree


def _bind(fn, args, kwargs):
    """Bind positional args to names so ops can be re-parameterised (clone(for_test)) and serialised."""
    try:
        sig = inspect.signature(fn)
    except (TypeError, ValueError):
        return args, kwargs
    if any(p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD) for p in sig.parameters.values()):
        return args, kwargs
    try:
        b = sig.bind(*args, **kwargs)
    except TypeError:
        return args, kwargs
    return (), dict(b.arguments)


# ----------------------------------------------------------------------------- InferMeta
# Shapes / dtypes of a recorded op come from running it on meta tensors (phi's InferMeta role).
# Two kinds of ops cannot run on meta tensors: ops whose output SIZE depends on input values
# (the second example run; reference: NonZeroInferMeta / UniqueRawInferMeta / MaskedSelectInferMeta / MultiClassNMSInferMeta
# give those dims -1, phi/infermeta/unary.cc:3377,3569, binary.cc:1489, multiary.cc) and ops that
# read a host value on the way (one_hot's range check, accuracy's counts, LoD offsets). For both the
# op runs once on small CPU EXAMPLE inputs of the recorded shapes (their output structure, dtypes
# and static dims), and for the data-dependent ones a second run on other example values marks the
# dims that moved as -1. The recorded op itself runs the real function at Executor.run time.
_INFER_META = {}          # op name -> fn(*meta args, **meta kwargs) -> meta outputs
_DATA_DEPENDENT = {"nonzero", "unique", "unique_consecutive", "masked_select", "where_index", "where",
                   "multiclass_nms", "multiclass_nms2", "multiclass_nms3", "matrix_nms", "locality_aware_nms",
                   "edit_distance", "ctc_align", "ctc_greedy_decoder", "generate_proposals", "distribute_fpn_proposals",
                   "collect_fpn_proposals", "box_decoder_and_assign", "detection_output", "retinanet_detection_output",
                   "sequence_erase", "sequence_enumerate", "filter_by_instag", "shuffle_batch", "tdm_sampler",
                   "masked_scatter", "bincount", "histogram_dd", "segment_sum", "segment_mean", "segment_max",
                   "segment_min", "unique_with_counts", "sample_neighbors", "graph_reindex", "graph_khop_sampler"}


def register_infer_meta(*names):
    """``@register_infer_meta("op")``: an explicit InferMeta for a recorded op (called with the
    op's arguments, Variables as meta tensors; returns the outputs as meta tensors)"""
    def deco(f):
        for n in names:
            _INFER_META[n] = f
        return f
    return deco


@register_infer_meta("print", "Print")
def _print_meta(x, *a, **k):   # the print op returns its input: nothing to run (or print) at build time
    return x


def _meta_unsupported(e):
    if isinstance(e, NotImplementedError):
        return True
    msg = str(e)
    return isinstance(e, (RuntimeError, ValueError, TypeError, IndexError)) and any(
        k in msg for k in ("meta", "Meta", "has no value", "no data", "data-dependent", "DataDependent"))


def _example(tree, dense, memo):
    """CPU example values for an InferMeta run. ``dense`` True: floats (1..n)/(n+1) (distinct,
    inside (0, 1)), integers zeros (valid indices / labels), bools True; False: all zeros / False;
    "mixed": floats cycling -1, 0, 1, integers 0, 1, bools alternating (the probe run of a
    data-dependent op, so comparisons and masks inside it see both outcomes)"""
    if isinstance(tree, Variable):
        k = id(tree)
        if k not in memo:
            m = tree._t
            n = max(int(m.numel()), 1)
            mixed = isinstance(dense, str)
            if m.dtype.is_floating_point or m.dtype.is_complex:
                if mixed:
                    t = (torch.arange(n) % 3 - 1).to(m.dtype)
                else:
                    t = (torch.arange(1, n + 1, dtype=torch.float64) / (n + 1)).to(m.dtype) if dense else \
                        torch.zeros(n, dtype=m.dtype)
                t = t[:m.numel()].reshape(m.shape)
            elif m.dtype == torch.bool:
                t = (torch.arange(n) % 2 == 0)[:m.numel()].reshape(m.shape) if mixed else torch.full(m.shape, bool(dense))
            else:
                t = (torch.arange(n) % 2).to(m.dtype)[:m.numel()].reshape(m.shape) if mixed else \
                    torch.zeros(m.shape, dtype=m.dtype)
            v = _wrap(t)
            lvl = getattr(tree, "lod_level", 0)
            if lvl and t.dim():      # a LoD feed: one sequence per level over all rows
                v._lod = [[0, int(t.shape[0])] for _ in range(lvl)]
            memo[k] = v
        return memo[k]
    if isinstance(tree, Tensor):
        if tree._t.device.type == "meta":
            return _wrap(torch.zeros(tree._t.shape, dtype=tree._t.dtype))
        # a captured parameter / persistable state: a CPU copy, so an op that updates its state in
        # place (auc's stat buffers, batch_norm's running moments) leaves the real one untouched
        if id(tree) not in memo:
            c = _wrap(tree._t.detach().to("cpu", copy=True))
            if getattr(tree, "_lod", None):
                c._lod = tree._lod
            memo[id(tree)] = c
        return memo[id(tree)]
    if isinstance(tree, list):
        return [_example(t, dense, memo) for t in tree]
    if isinstance(tree, tuple):
        return tuple(_example(t, dense, memo) for t in tree)
    if isinstance(tree, dict):
        return {k: _example(v, dense, memo) for k, v in tree.items()}
    return tree


def _meta_of(tree):
    if isinstance(tree, Tensor):
        return _wrap(tree._t.detach().to("meta"))
    if isinstance(tree, torch.Tensor):
        return _wrap(tree.detach().to("meta"))
    if isinstance(tree, list):
        return [_meta_of(t) for t in tree]
    if isinstance(tree, tuple):
        return tuple(_meta_of(t) for t in tree)
    return tree


def _run_example(fn, bargs, bkw, dense):
    """the op on example inputs, with the default device switched to the CPU for the call (the
    ops' own allocations land beside the examples)"""
    memo = {}
    prev = _core._default_device
    _core._default_device = torch.device("cpu")
    try:
        with torch.no_grad():
            return fn(*_example(bargs, dense, memo), **_example(bkw, dense, memo))
    finally:
        _core._default_device = prev


def _infer_meta(fn, name, bargs, bkw):
    """-> (meta outputs, dynamic dims per output tensor or None)"""
    _core._mode.record_depth += 1
    try:
        f = _INFER_META.get(name)
        if f is not None:
            return f(*_to_meta(bargs), **_to_meta(bkw)), None
        try:
            return fn(*_to_meta(bargs), **_to_meta(bkw)), None
        except Exception as e:   # noqa: BLE001 - classified below
            if not _meta_unsupported(e):
                raise
        out = _run_example(fn, bargs, bkw, True)
        dyn = None
        if name in _DATA_DEPENDENT:
            a = list(_iter_tensors(out if isinstance(out, (list, tuple)) else [out]))
            moved = [set() for _ in a]
            for mode in (False, "mixed"):
                try:
                    other = _run_example(fn, bargs, bkw, mode)
                except Exception:   # noqa: BLE001 - the other examples are only probes
                    continue
                b = list(_iter_tensors(other if isinstance(other, (list, tuple)) else [other]))
                if len(a) != len(b):
                    continue
                for mv, ta, tb in zip(moved, a, b):
                    if ta._t.dim() == tb._t.dim():
                        mv.update(i for i, (x, y) in enumerate(zip(ta._t.shape, tb._t.shape)) if x != y)
            dyn = [tuple(sorted(mv)) for mv in moved]
        return _meta_of(out), dyn
    finally:
        _core._mode.record_depth -= 1


_PROBE = 7   # the size a -1 dim takes in the second meta run (the first uses 1)


def _dynamic_dims(v):
    ds = v.declared_shape
    if ds is None or len(ds) != v._t.dim():
        return ()
    return tuple(i for i, d in enumerate(ds) if d is not None and d < 0)


def _to_probe(tree, size=_PROBE):
    if isinstance(tree, Variable):
        dims = _dynamic_dims(tree)
        if not dims:
            return _wrap(tree._t)
        shp = [size if i in dims else int(s) for i, s in enumerate(tree._t.shape)]
        return _wrap(torch.empty(shp, dtype=tree._t.dtype, device="meta"))
    if isinstance(tree, list):
        return [_to_probe(t, size) for t in tree]
    if isinstance(tree, tuple):
        return tuple(_to_probe(t, size) for t in tree)
    if isinstance(tree, dict):
        return {k: _to_probe(v, size) for k, v in tree.items()}
    return _to_meta(tree)


def _infer_meta_dynamic(fn, bargs, bkw):
    """InferMeta for an op that rejects the size-1 stand-in of a -1 dim (BatchNorm training at a
    1 x 1 map: "more than 1 value per channel", instance / group statistics ...). The reference's
    InferMeta is shape-only (phi/infermeta/multiary.cc:437) and never sees a value; here the op
    runs on meta inputs whose -1 dims take two probe sizes, the output dims that follow them
    become -1 (stored as 1, as every -1 dim of a recorded Variable) and the rest are static.
    None when no input has a -1 dim or a probe fails too."""
    if not any(_dynamic_dims(v) for v in _iter_vars((bargs, bkw))):
        return None
    _core._mode.record_depth += 1
    try:
        a = fn(*_to_probe(bargs, _PROBE), **_to_probe(bkw, _PROBE))
        b = fn(*_to_probe(bargs, _PROBE + 6), **_to_probe(bkw, _PROBE + 6))
    except Exception:   # noqa: BLE001 - the original error is raised by the caller
        return None
    finally:
        _core._mode.record_depth -= 1
    ta = list(_iter_tensors(a if isinstance(a, (list, tuple)) else [a]))
    tb = list(_iter_tensors(b if isinstance(b, (list, tuple)) else [b]))
    if len(ta) != len(tb):
        return None
    dyn = []
    for x, y in zip(ta, tb):
        d = tuple(i for i, (p, q) in enumerate(zip(x._t.shape, y._t.shape)) if p != q) \
            if x._t.dim() == y._t.dim() else ()
        dyn.append(d)
        if d:   # the -1 dims' stand-in size 1, in place
            x._t = torch.empty([1 if i in d else int(n) for i, n in enumerate(x._t.shape)], dtype=x._t.dtype,
                               device="meta")
    return _meta_of(a), dyn


def _propagate_dynamic(fn, bargs, bkw, meta_out):
    """-1 dims through an op: a second meta run with the inputs' -1 dims at another size; the
    output dims that move with it are -1 (a -1 batch stays -1 through the layers, as the
    reference's InferMeta keeps it). None when no input has a -1 dim or the probe fails."""
    if not any(_dynamic_dims(v) for v in _iter_vars((bargs, bkw))):
        return None
    _core._mode.record_depth += 1
    try:
        probe = fn(*_to_probe(bargs), **_to_probe(bkw))
    except Exception:   # noqa: BLE001 - e.g. a reshape to fixed dims: the output stays static
        return None
    finally:
        _core._mode.record_depth -= 1
    a = list(_iter_tensors(meta_out if isinstance(meta_out, (list, tuple)) else [meta_out]))
    b = list(_iter_tensors(probe if isinstance(probe, (list, tuple)) else [probe]))
    if len(a) != len(b):
        return None
    return [tuple(i for i, (x, y) in enumerate(zip(ta._t.shape, tb._t.shape)) if x != y)
            if ta._t.dim() == tb._t.dim() else () for ta, tb in zip(a, b)]


def _mark_dynamic(outs, dyn):
    if not dyn:
        return
    for v, dims in zip(_iter_vars(outs), dyn):
        if dims:
            v.declared_shape = [-1 if i in dims else int(s) for i, s in enumerate(v._t.shape)]


def record_op(fn, name, args, kwargs):
    """Called by every wrapped op in static mode (see framework/dispatch.py)."""
    if not _has_var((args, kwargs)):
        return fn(*args, **kwargs)
    qual = f"{fn.__module__}.{name}"
    OP_REGISTRY.setdefault(qual, fn)
    bargs, bkw = _bind(fn, args, kwargs)
    try:
        meta_out, dyn = _infer_meta(fn, name, bargs, bkw)
    except Exception:
        r = _infer_meta_dynamic(fn, bargs, bkw)
        if r is None:
            raise
        meta_out, dyn = r
    if dyn is None and os.environ.get("PHA_STATIC_DYN_DIMS", "1") != "0":
        dyn = _propagate_dynamic(fn, bargs, bkw, meta_out)
    blk = default_main_program().current_block()
    outs = _outputs_to_vars(meta_out, blk)
    _mark_dynamic(outs, dyn)
    op = OpDesc(qual, fn, bargs, bkw, outs)
    if _OP_DEVICE[0] is not None:     # static.device_guard: pipeline stage / placement of the op
        op.attrs["op_device"] = _OP_DEVICE[0]
    for v in _iter_vars(outs):
        v.op = op
    blk.append_op(op)
    return outs


_OP_DEVICE = [None]


def set_ref_op(outs, typ, ins, routs, attrs):
    """attach the reference op form (type, {slot: [tensors]} in / out, attributes) to the recorded op
    that produced ``outs``: serialize_program / save_inference_model write it under that type and
    the reader's converter (static/ref_ops.py) maps it back. No-op outside a static Program."""
    v = next(_iter_vars(outs if isinstance(outs, (list, tuple)) else [outs]), None)
    if v is None or getattr(v, "op", None) is None:
        return
    v.op.attrs["ref_op"] = (typ, {k: list(t) for k, t in ins.items() if t and t[0] is not None},
                            {k: list(t) for k, t in routs.items() if t and t[0] is not None}, dict(attrs))


# ----------------------------------------------------------------------------- backward / optimize ops
def _grad_var(block, like, name):
    v = Variable(block, like._t.to("meta") if like._t.device.type != "meta" else like._t, name)
    block.vars[name] = v
    return v


def is_train_op(op):
    """a backward / loss-grad / optimizer op (not part of an inference program)"""
    return op.type.startswith("@") or op.attrs.get("op_role") in ("backward", "optimize", "loss")


def append_backward(loss, parameter_list=None, no_grad_set=None, callbacks=None, checkpoints=None,
                    distop_context=None):
    """per-op backward (static/backward.py)"""
    from .backward import append_backward as _ab
    return _ab(loss, parameter_list, no_grad_set, callbacks, checkpoints, distop_context)


def _append_backward_opaque(loss, parameter_list=None, no_grad_set=None, callbacks=None, checkpoints=None,
                            distop_context=None):
    prog = default_main_program()
    blk = prog.global_block()
    params = parameter_list if parameter_list is not None else [p for p in prog.all_parameters() if p.trainable]
    params = [blk.vars.get(p, p) if isinstance(p, str) else p for p in params]
    nog = set(id(v) for v in (no_grad_set or []) if not isinstance(v, str))
    params = [p for p in params if id(p) not in nog]
    gvars = [_grad_var(blk, p, p.name + "@GRAD") for p in params]

    def _backward(loss_t, *ps):
        grads = torch.autograd.grad(loss_t._t, [p._t for p in ps], allow_unused=True, retain_graph=True)
        return tuple(_wrap(g if g is not None else torch.zeros_like(p._t)) for g, p in zip(grads, ps))

    op = OpDesc("@backward", _backward, (loss,) + tuple(params), {}, tuple(gvars))
    blk.append_op(op)
    return list(zip(params, gvars))


def gradients(targets, inputs, target_gradients=None, no_grad_set=None):
    from .backward import gradients as _g
    return _g(targets, inputs, target_gradients, no_grad_set)


def _gradients_opaque(targets, inputs, target_gradients=None, no_grad_set=None):
    prog = default_main_program()
    blk = prog.global_block()
    targets = [targets] if isinstance(targets, Tensor) else list(targets)
    inputs = [inputs] if isinstance(inputs, Tensor) else list(inputs)
    for v in inputs:
        if isinstance(v, Variable):
            v.need_grad = True
    tg = target_gradients if target_gradients is None or isinstance(target_gradients, (list, tuple)) else [target_gradients]
    gvars = [_grad_var(blk, x, x.name + "@GRAD") for x in inputs]

    def _grads(ts, xs, gts):
        gs = torch.autograd.grad([t._t for t in ts], [x._t for x in xs], [g._t for g in gts] if gts else None,
                                 allow_unused=True, retain_graph=True, create_graph=True)
        return tuple(_wrap(g if g is not None else torch.zeros_like(x._t)) for g, x in zip(gs, xs))

    op = OpDesc("@gradients", _grads, (tuple(targets), tuple(inputs), tuple(tg or ())), {}, tuple(gvars))
    blk.append_op(op)
    return gvars


def minimize_static(optimizer, loss, parameters=None, no_grad_set=None):
    from .backward import minimize as _m
    return _m(optimizer, loss, parameters, no_grad_set)


def _minimize_opaque(optimizer, loss, parameters=None, no_grad_set=None):
    prog = default_main_program()
    blk = prog.global_block()
    params = parameters if parameters is not None else [p for p in prog.all_parameters() if p.trainable]
    nog = set(id(v) for v in (no_grad_set or []) if not isinstance(v, str))
    params = [p for p in params if id(p) not in nog]
    if optimizer._parameter_list is None:
        optimizer._add_param_group({"params": list(params)})
        optimizer._parameter_list = list(params)
    gvars = [_grad_var(blk, p, p.name + "@GRAD") for p in params]

    def _optimize(loss_t, *ps):
        for p in ps:
            p._t.grad = None
        loss_t._t.backward()
        grads = tuple(_wrap(p._t.grad if p._t.grad is not None else torch.zeros_like(p._t)) for p in ps)
        with _core_dynamic():
            optimizer.step()
        optimizer.clear_grad(set_to_zero=False)
        return grads

    op = OpDesc("@optimize", _optimize, (loss,) + tuple(params), {}, tuple(gvars))
    blk.append_op(op)
    return [op], list(zip(params, gvars))


@contextlib.contextmanager
def _core_dynamic():
    prev = _core._mode.static
    _core._mode.static = False
    try:
        yield
    finally:
        _core._mode.static = prev


# ----------------------------------------------------------------------------- scope / executor
class _TensorView:
    """``scope.find_var(name).get_tensor()``: a LoDTensor handle onto the scope's value (reference
    pybind tensor_py.h). ``set(array, place)`` writes INTO the held tensor when the shape and dtype
    match — every program reading that parameter sees the new value at its next run — and
    otherwise rebinds it."""

    def __init__(self, holder):
        self._h = holder

    @property
    def _v(self):
        return self._h.value

    def set(self, array, place=None):
        arr = np.ascontiguousarray(array.numpy() if isinstance(array, Tensor) else np.asarray(array))
        t = self._v
        dev = _core._to_torch_device(place) if place is not None else (
            t._t.device if t is not None and t._t.device.type != "meta" else _core.default_device())
        new = torch.from_numpy(arr).to(dev)
        if t is None:
            self._h.value = _wrap(new)
            return
        with torch.no_grad():
            if tuple(t._t.shape) == tuple(new.shape) and t._t.device == new.device:
                t._t.copy_(new.to(t._t.dtype))
            else:
                t._t = new.to(t._t.dtype) if t._t.dtype.is_floating_point == new.dtype.is_floating_point else new

    def __array__(self, dtype=None, copy=None):
        # always a copy: the CPU tensor's numpy() would alias the live parameter memory
        a = self._v._t.detach().cpu().numpy().copy() if self._v is not None else np.zeros([0], "float32")
        return a.astype(dtype) if dtype is not None else a

    def numpy(self):
        return np.asarray(self)

    def shape(self):
        return list(self._v._t.shape) if self._v is not None else []

    def _dtype(self):
        return self._v._t.dtype if self._v is not None else None

    def lod(self):
        return [list(l) for l in (getattr(self._v, "_lod", None) or [])]

    def set_lod(self, lod):
        self._v._lod = [list(map(int, l)) for l in lod]

    def recursive_sequence_lengths(self):
        return [[b - a for a, b in zip(l[:-1], l[1:])] for l in self.lod()]

    def set_recursive_sequence_lengths(self, lengths):
        self.set_lod([list(np.concatenate([[0], np.cumsum(l)]).astype(int)) for l in lengths])

    def _is_initialized(self):
        return self._v is not None

    def __repr__(self):
        return f"LoDTensor(shape={self.shape()}, lod={self.lod()})"


class _ScopeVar:
    def __init__(self, name, value=None):
        self.name, self.value = name, value

    def get_tensor(self):
        return _TensorView(self)

    def is_initialized(self):
        return self.value is not None

    def set(self, value, place=None):
        self.get_tensor().set(value, place)


# every persistable tensor a static Program created or ran (parameters, optimizer accumulators,
# metric statistics) by name: what the root scope resolves names to
_PERSISTABLES = weakref.WeakValueDictionary()


def register_persistable(t):
    n = getattr(t, "name", None)
    if n:
        _PERSISTABLES[n] = t


class Scope:
    """Holds the values of a Program's persistable variables (reference framework/scope.h,
    fluid/executor.py:47). The root scope holds the tensors the Program was built with
    (parameters are initialised when they are created); another scope holds its own copies:
    ``Executor.run(startup, scope=s)`` initialises fresh parameters in ``s`` with their
    initializers, and ``Executor.run(main, scope=s)`` reads and updates ``s``'s values (persistables
    ``s`` lacks are copied in from the root at first use), so two scopes train independently.
    Child scopes (``new_scope``) see their parents' variables."""

    def __init__(self, parent=None, _root=False):
        self.vars = {}
        self._parent = parent
        self._kids = []
        self._root = _root

    def var(self, name):
        v = self.find_var(name)
        if v is None:
            v = self.vars[name] = _ScopeVar(name)
            v.user = True   # created by the user: its value seeds a same-named persistable
        return v

    def find_var(self, name):
        v = self.vars.get(name)
        if v is None and self._root:
            t = _PERSISTABLES.get(name)
            if t is not None:
                v = self.vars[name] = _ScopeVar(name, t)
        if v is None and self._parent is not None:
            return self._parent.find_var(name)
        return v

    def find_local_var(self, name):
        return self.vars.get(name)

    def new_scope(self):
        c = Scope(self)
        self._kids.append(c)
        return c

    def drop_kids(self):
        self._kids = []

    def kids(self):
        return list(self._kids)

    def local_var_names(self):
        return list(self.vars)

    def erase(self, names):
        for n in names:
            self.vars.pop(n, None)

    def _bind(self, t):
        """the value this scope holds for the persistable tensor ``t`` (created here from ``t`` when
        missing: the root scope holds ``t`` itself, other scopes a copy)"""
        name = getattr(t, "name", None)
        if not name:
            return t
        if self._root:
            # the root scope IS the build-time tensors: several programs (a loaded copy of a
            # program, say) may each hold their own tensor under one name. A value the user put
            # under the name before the first run (var(name).get_tensor().set) is taken over.
            v = self.vars.get(name)
            if v is not None and getattr(v, "user", False) and v.value is not None and v.value is not t and \
                    tuple(v.value._t.shape) == tuple(t._t.shape):
                with torch.no_grad():
                    t._t.copy_(v.value._t.to(t._t.device, t._t.dtype))
            self.vars[name] = _ScopeVar(name, t)
            _PERSISTABLES[name] = t
            return t
        v = self.find_var(name)
        if v is None or v.value is None:
            val = t if self._root else (Parameter(data=t._t.detach().clone(), name=name, trainable=t.trainable)
                                       if isinstance(t, Parameter) else _named_clone(t))
            if v is None:
                v = self.vars[name] = _ScopeVar(name, val)
            else:
                v.value = val
        return v.value


def _named_clone(t):
    c = _wrap(t._t.detach().clone())
    c.name = t.name
    c.persistable = getattr(t, "persistable", True)
    return c


_global_scope = Scope(_root=True)


def global_scope():
    return _global_scope


@contextlib.contextmanager
def scope_guard(scope):
    global _global_scope
    old = _global_scope
    _global_scope = scope
    try:
        yield
    finally:
        _global_scope = old


def _scope_overrides(program, scope):
    """{id(build-time tensor): the scope's value} for every persistable the program touches"""
    over = {}
    for t in _program_tensors(program):
        if not (isinstance(t, Parameter) or getattr(t, "persistable", False)):
            continue
        v = scope._bind(t)
        if v is not t:
            over[id(t)] = v
    return over


class _RunScope(threading.local):   # the scope of the Executor.run in progress (per thread)
    def __init__(self):
        self.v = None

    def __getitem__(self, i):
        return self.v

    def __setitem__(self, i, v):
        self.v = v


_RUN_SCOPE = _RunScope()


_OPT_LOCKS = {}
_OPT_LOCKS_GUARD = threading.Lock()


def optimizer_lock(opt):
    """the lock that serialises one optimizer's updates across dataset-trainer threads"""
    with _OPT_LOCKS_GUARD:
        return _OPT_LOCKS.setdefault(id(opt), threading.RLock())


@contextlib.contextmanager
def scoped_optimizer(opt, originals, values):
    """an optimizer op running in a non-root scope: the step updates the scope's parameter copies
    with the scope's own optimizer state (accumulators, master weights, step count)"""
    sc = _RUN_SCOPE[0]
    if sc is None or all(a is b for a, b in zip(originals, values)):
        yield
        return
    st = sc.__dict__.setdefault("_opt_states", {}).setdefault(id(opt), {
        "_accumulators": collections.defaultdict(dict), "_master_weights": {}, "_step_count": 0, "_pstep": {}})
    saved = {k: getattr(opt, k, None) for k in st}
    groups = [list(g["params"]) for g in opt._param_groups]
    plist = opt._parameter_list
    swap = {id(a): b for a, b in zip(originals, values)}
    try:
        for k, v in st.items():
            setattr(opt, k, v)
        for g in opt._param_groups:
            g["params"] = [swap.get(id(q), q) for q in g["params"]]
        opt._parameter_list = [swap.get(id(q), q) for q in (plist or [])]
        yield
    finally:
        for k in st:
            st[k] = getattr(opt, k)
            setattr(opt, k, saved[k])
        for g, ps in zip(opt._param_groups, groups):
            g["params"] = ps
        opt._parameter_list = plist


def _init_in_scope(startup, scope):
    """the startup program run in ``scope``: fresh parameters from their initializers"""
    if scope._root:
        return
    for p, init in startup.__dict__.get("_param_inits", ()):
        q = Parameter(list(p._t.shape), p._t.dtype, name=p.name, trainable=p.trainable)
        if init is not None:
            init(q)
        else:
            q._t.data.copy_(p._t)
        v = scope.vars.get(p.name)
        if v is None:
            scope.vars[p.name] = _ScopeVar(p.name, q)
        else:
            v.value = q


def note_parameter(p, init):
    """a parameter created in a static Program: the startup program re-runs ``init`` for another
    scope, and the root scope resolves its name"""
    if not _core._mode.static:
        return
    register_persistable(p)
    default_startup_program().__dict__.setdefault("_param_inits", []).append((p, init))


def _subst(tree, env):
    if isinstance(tree, Variable):
        try:
            return env[id(tree)]
        except KeyError:
            raise RuntimeError(f"variable {tree.name} has no value (missing feed?)")
    if isinstance(tree, Tensor):   # a persistable: the running scope's value (Scope._bind)
        return env.get(id(tree), tree)
    if isinstance(tree, list):
        return [_subst(t, env) for t in tree]
    if isinstance(tree, tuple):
        return tuple(_subst(t, env) for t in tree)
    if isinstance(tree, dict):
        return {k: _subst(v, env) for k, v in tree.items()}
    return tree


def _bind_outputs(outs, vals, env):
    if isinstance(outs, Variable):
        env[id(outs)] = vals
    elif isinstance(outs, (list, tuple)):
        for o, v in zip(outs, vals):
            _bind_outputs(o, v, env)


_SUB_BLOCK_ATTRS = ("true_block", "false_block", "cond_block", "body_block", "sub_block")


def _op_uses(program, op):
    """ids of the Variables ``op`` may read: its inputs, and for a control-flow op every Variable
    named in its attributes or read by any op of its sub-blocks (conservative)"""
    ids = {id(v) for v in _iter_vars((op.args, op.kwargs))}
    if op.exec is not None:
        ids |= {id(v) for v in _iter_vars(list(op.attrs.values()))}
        for k in _SUB_BLOCK_ATTRS:
            b = op.attrs.get(k)
            if isinstance(b, int) and 0 <= b < len(program.blocks):
                for sop in program.blocks[b].ops:
                    ids |= _op_uses(program, sop)
    return ids


def _lifetimes(program, blk, keep_ids):
    """(first definition op, last use op) of every Variable of ``blk``'s top-level ops; Variables
    in ``keep_ids`` (fetch targets) never end"""
    first, last = {}, {}
    for i, op in enumerate(blk.ops):
        for vid in _op_uses(program, op):
            last[vid] = i
            first.setdefault(vid, -1)      # defined before the block (feed) unless seen below
        for v in _iter_vars(op.outputs):
            first.setdefault(id(v), i)
            last.setdefault(id(v), i)
    for vid in keep_ids:
        if vid in last:
            last[vid] = len(blk.ops)
    return first, last


def _gc_plan(program, blk, fetch_ids):
    """eager deletion (reference framework/ir/memory_optimize_pass/eager_deletion_pass, the
    InterpreterCore garbage collector): op index -> Variable ids whose last reader it is. Cached per
    (op count, fetch set)."""
    key = (len(blk.ops), tuple(sorted(fetch_ids)))
    cache = program.__dict__.setdefault("_gc_cache", {})
    plan = cache.get(key)
    if plan is None:
        _, last = _lifetimes(program, blk, fetch_ids)
        plan = {}
        for vid, i in last.items():
            if i < len(blk.ops):
                plan.setdefault(i, []).append(vid)
        cache[key] = plan
    return plan


def plan_program_memory(program, fetch_list=(), alignment=256):
    """Static memory plan of the global block from the Variables' inferred shapes and their
    lifetimes, on the native best-fit planner (csrc/runtime/arena.cpp): returns
    {"arena_bytes": planned peak with buffer reuse, "naive_bytes": every intermediate kept,
    "offsets": {name: byte offset}} — what the eager deletion above frees in practice."""
    from ..utils import native
    blk = program.global_block()
    fetch_ids = {id(blk.vars[f]) if isinstance(f, str) else id(f) for f in fetch_list}
    first, last = _lifetimes(program, blk, fetch_ids)
    by_id = {}
    for op in blk.ops:
        for v in _iter_vars((op.args, op.kwargs, op.outputs)):
            by_id[id(v)] = v
    names, sizes, f, e = [], [], [], []
    for vid, v in by_id.items():
        t = v._t
        if t is None or not hasattr(t, "numel") or v.persistable:
            continue
        names.append(v.name)
        sizes.append(max(1, int(t.numel()) * t.element_size()))
        f.append(max(0, first.get(vid, 0)))
        e.append(max(f[-1], last.get(vid, f[-1])))
    if not names:
        return {"arena_bytes": 0, "naive_bytes": 0, "offsets": {}}
    offs, total = native.plan_memory(sizes, f, e, alignment)
    return {"arena_bytes": total, "naive_bytes": int(sum(sizes)), "offsets": dict(zip(names, offs))}


def _program_tensors(program):
    """the real (persistable) tensors the program's ops read or write"""
    seen, out = set(), []
    for op in (o for b in program.blocks for o in b.ops):
        for t in _iter_tensors((op.args, op.kwargs, op.outputs)):
            if not isinstance(t, Variable) and id(t) not in seen:
                seen.add(id(t))
                out.append(t)
    return out


def run_program(program, feed, fetch_list, scope=None):
    """Interpret ``program`` with ``feed``; returns fetched Tensors (real). Intermediate values are
    dropped right after their last reader (eager deletion). Persistables read and write ``scope``'s
    values (default: the root scope, i.e. the tensors the program was built with)."""
    blk = program.global_block()
    sc = scope if scope is not None else _global_scope
    env = _scope_overrides(program, sc)
    prev_scope, _RUN_SCOPE[0] = _RUN_SCOPE[0], (sc if env else None)
    from .trainer import hogwild_alias
    if hogwild_alias():
        for t in _program_tensors(program):
            if isinstance(t, Parameter) and id(t) not in env and t._t.is_floating_point():
                a = _wrap(t._t.data)   # same storage, own version counter
                a._t.requires_grad_(t._t.requires_grad)
                a.name, a.persistable, a._hogwild_of = t.name, True, t
                env[id(t)] = a
    try:
        return _run_program(program, blk, env, feed, fetch_list)
    finally:
        _RUN_SCOPE[0] = prev_scope


def _run_program(program, blk, env, feed, fetch_list):
    for name, val in (feed or {}).items():
        v = blk.vars.get(name)
        if v is None:
            continue
        t = val._t if isinstance(val, Tensor) else _core._to_torch(np.asarray(val) if not isinstance(val, torch.Tensor) else val,
                                                                    dtype=v._t.dtype)
        if t.dtype != v._t.dtype:
            t = t.to(v._t.dtype)
        if t.device != _core.default_device():
            t = t.to(_core.default_device())
        if v.need_grad and t.is_floating_point():
            t = t.detach().requires_grad_(True)
        env[id(v)] = _wrap(t)
        if getattr(val, "_lod", None):      # fluid LoD tensors keep their sequence offsets
            env[id(v)]._lod = val._lod
            program.__dict__["_lod_run"] = True   # outputs share their inputs' LoD (_share_lod)
    fetch_ids = set()
    for f in fetch_list or []:
        if isinstance(f, str) and f in blk.vars:
            fetch_ids.add(id(blk.vars[f]))
        elif isinstance(f, Variable):
            fetch_ids.add(id(f))
    free = _gc_plan(program, blk, fetch_ids) if os.environ.get("PHA_EAGER_DELETE", "1") != "0" else None
    prev_static = _core._mode.static
    _core._mode.record_depth += 1
    try:
        run_block(program, blk, env, free)
    finally:
        _core._mode.record_depth -= 1
        _core._mode.static = prev_static
    res = []
    for f in fetch_list or []:
        if isinstance(f, str):
            if f not in blk.vars:   # a persistable (parameter / optimizer state) by name
                hit = [env.get(id(t), t) for t in _program_tensors(program) if getattr(t, "name", None) == f]
                if not hit:
                    raise KeyError(f)
                res.append(_wrap(hit[0]._t.detach().clone()))   # a snapshot: later steps update it in place
                continue
            f = blk.vars[f]
        if isinstance(f, Variable):
            res.append(env[id(f)])
        elif isinstance(f, Tensor):
            res.append(env.get(id(f), f))
        else:
            raise TypeError(f"cannot fetch {f!r}")
    return res


def _cut_inputs(op, env):
    """A forward op that has a grad op (static/backward.py) reads its non-leaf inputs as fresh
    autograd leaves (detached views), kept in ``env`` under ("leaf", id(op), id(var)): the grad
    op's vector-Jacobian product then covers exactly this op's own computation — without the cut,
    an input that also reaches the op through another input (y = f(x) + x) would be differentiated
    along both paths here and again in f's grad op."""
    saved = {}
    for v in _iter_vars((op.args, op.kwargs)):
        val = env.get(id(v))
        if isinstance(val, Tensor) and val._t.requires_grad and val._t.grad_fn is not None and id(v) not in saved:
            leaf = _wrap(val._t.detach().requires_grad_(True))
            if getattr(val, "_lod", None):
                leaf._lod = val._lod
            saved[id(v)] = val
            env[id(v)] = leaf
            env[("leaf", id(op), id(v))] = leaf
    return saved


def _grad_env(op, env):
    """the value environment a grad op reads: its forward op's cut leaves in place of the inputs"""
    fid = op.attrs.get("_fwd_id")
    if fid is None:
        return env
    ins = op.kwargs.get("ins", ())
    over = {}
    for v in _iter_vars(ins):
        leaf = env.get(("leaf", fid, id(v)))
        if leaf is not None:
            over[id(v)] = leaf
    if not over:
        return env
    e2 = dict(env)
    e2.update(over)
    return e2


def _share_lod(op, out, env):
    """the reference's ShareLoD (InferShape ctx->ShareLoD("X", "Out")): an output that has no LoD
    of its own and keeps the row count of a LoD input carries that input's sequence offsets (fc,
    embedding, activations ... on fluid LoD tensors); the sequence ops set theirs themselves"""
    src = None
    for v in _iter_vars((op.args, op.kwargs)):
        val = env.get(id(v))
        lod = getattr(val, "_lod", None)
        if lod:
            src = (val._t.shape[0] if val._t.dim() else None, lod)
            break
    if src is None:
        return
    for t in _iter_tensors(out if isinstance(out, (list, tuple)) else [out]):
        if not getattr(t, "_lod", None) and t._t.dim() and t._t.shape[0] == src[0]:
            t._lod = src[1]


def run_block(program, blk, env, free=None):
    """interpret the ops of ``blk`` in the value environment ``env`` (Variable id -> Tensor);
    ``free``: op index -> Variable ids to drop after that op (eager deletion)"""
    cut_ids = program.__dict__.get("_cut_ops") or ()
    timer = program.__dict__.get("_op_timer")   # cost_model.profile_measure: per-op times
    for i, op in enumerate(blk.ops):
        if timer is not None:
            timer[1]()
            t_op = time.perf_counter()
        saved = _cut_inputs(op, env) if id(op) in cut_ids else None
        if op.exec is not None:
            op.exec(program, env, op)
        elif op.attrs.get("no_grad"):   # recompute segments: no autograd state kept in forward
            with torch.no_grad():
                out = op.fn(*_subst(op.args, env), **_subst(op.kwargs, env))
            # the values leave the segment as gradient-requiring leaves: ops after the last
            # checkpoint build their graph on them and their grad ops reach them
            for t in _iter_tensors(out if isinstance(out, (list, tuple)) else [out]):
                if t._t.is_floating_point() and not t._t.requires_grad:
                    t._t.requires_grad_(True)
            _bind_outputs(op.outputs, out, env)
        else:
            e = _grad_env(op, env) if "_fwd_id" in op.attrs else env
            out = op.fn(*_subst(op.args, e), **_subst(op.kwargs, e))
            _bind_outputs(op.outputs, out, env)
            if program.__dict__.get("_lod_run"):
                _share_lod(op, out, e)
        if saved:   # later readers see the original values (and their graph)
            env.update(saved)
        if timer is not None:
            timer[1]()
            timer[0].append((blk.idx, i, (time.perf_counter() - t_op) * 1e3))
        if free:
            for vid in free.get(i, ()):
                env.pop(vid, None)
    if free is not None:
        program.__dict__["_last_env_size"] = len(env)


def has_control_flow(program):
    return len(program.blocks) > 1 or any(op.exec is not None for op in program.global_block().ops)


_CLOSE_HOOKS = []


def register_close_hook(fn):
    """``fn()`` runs at the next ``Executor.close()`` (once)"""
    _CLOSE_HOOKS.append(fn)


class Executor:
    def __init__(self, place=None):
        self.place = place

    def run(self, program=None, feed=None, fetch_list=None, feed_var_name="feed", fetch_var_name="fetch",
            scope=None, return_numpy=True, use_program_cache=False, return_merged=True, use_prune=False):
        if program is None:
            program = default_main_program()
        # fluid py_reader / DataLoader.from_generator attached to the program: a run without an
        # explicit feed pulls the next batch (EOFException ends the pass)
        pipe = program.__dict__.get("_pipeline") if not isinstance(program, CompiledProgram) else None
        if pipe is not None:      # static pipeline parallelism: this rank's stage over micro-batches
            outs = pipe.run(feed or {}, fetch_list or [])
            return [o.numpy() if isinstance(o, Tensor) and return_numpy else o for o in outs]
        readers = [r for r in program.__dict__.get("_py_readers", ()) if getattr(r, "_it", None) is not None]
        if readers and not feed:
            feed = {}
            for r in readers:
                feed.update(r._next_feed())
        if isinstance(program, CompiledProgram):
            outs = program._run(feed, fetch_list, scope)
        else:
            sc = scope if scope is not None else _global_scope
            if program.__dict__.get("_param_inits"):
                _init_in_scope(program, sc)
            if not program.global_block().ops:
                return []
            outs = run_program(program, feed, fetch_list, sc)
        if return_numpy:
            return [o.numpy() if isinstance(o, Tensor) else o for o in outs]
        return outs

    def close(self):
        """end this process' part in a distributed job: the close hooks registered by the
        transpiled programs run (a DistributeTranspiler trainer leaves the parameter servers)"""
        while _CLOSE_HOOKS:
            _CLOSE_HOOKS.pop(0)()

    def train_from_dataset(self, program=None, dataset=None, scope=None, thread=0, debug=False, fetch_list=None,
                           fetch_info=None, print_period=100, fetch_handler=None):
        """``thread`` Hogwild (or, for a parameter-server program, DownpourSGD) worker threads over
        the dataset's batches (static/trainer.py)"""
        from .trainer import run_from_dataset
        return run_from_dataset(self, program, dataset, scope, thread, False, debug, fetch_list, fetch_info,
                                print_period, fetch_handler)

    def infer_from_dataset(self, program=None, dataset=None, scope=None, thread=0, debug=False, fetch_list=None,
                           fetch_info=None, print_period=100, fetch_handler=None):
        """the program's inference part (backward / optimizer ops dropped) over the dataset"""
        from .trainer import run_from_dataset
        return run_from_dataset(self, program, dataset, scope, thread, True, debug, fetch_list, fetch_info,
                                print_period, fetch_handler)


class BuildStrategy:
    def __init__(self):
        self.fuse_elewise_add_act_ops = False
        self.fuse_bn_act_ops = False
        self.fuse_all_reduce_ops = True
        self.enable_inplace = True
        self.enable_addto = False
        self.memory_optimize = True
        self.fuse_gemm_epilogue = True
        self.use_hip_graph = False
        self.build_cinn_pass = False
        self.sync_batch_norm = False
        self.reduce_strategy = 0
        self.gradient_scale_strategy = 0
        self.debug_graphviz_path = ""


class ExecutionStrategy:
    def __init__(self):
        self.num_threads = 1
        self.num_iteration_per_drop_scope = 100
        self.use_thread_barrier = False


def data_parallel_program(program, world, bucket_bytes=64 << 20):
    """insert the bucketed, backward-overlapped gradient all-reduce (mean over ``world`` ranks) in
    front of ``program``'s optimizer ops, in place; a program already rewritten is left alone"""
    if program.__dict__.get("_dp_world"):
        return program
    from ..parallel.fleet.static_optimizers import StaticFleetOptimizer
    blk = program.global_block()
    opt_ops = [op for op in blk.ops if op.attrs.get("op_role") in ("optimize", 2) and "grads" in op.kwargs]
    if not opt_ops:
        program.__dict__["_dp_world"] = world
        return program
    for op in opt_ops:
        blk.ops.remove(op)
    helper = StaticFleetOptimizer.__new__(StaticFleetOptimizer)
    helper.world = world
    grads = [g for op in opt_ops for g in op.kwargs["grads"]]
    reduced = helper._insert_overlapped_allreduce(blk, grads, bucket_bytes, world=world)
    k = 0
    for op in opt_ops:
        n = len(op.kwargs["grads"])
        op.kwargs = dict(op.kwargs, grads=tuple(reduced[k:k + n]))
        k += n
        blk.append_op(op)
    program.__dict__["_dp_world"] = world
    return program


class CompiledProgram:
    """Program + build strategy. With ``build_strategy.use_hip_graph`` a forward-only program is
    captured once per feed signature into a HIP graph and replayed (static input/output
    buffers), removing per-op launch overhead."""

    def __init__(self, program_or_graph, build_strategy=None):
        self._program = program_or_graph
        self._build_strategy = build_strategy or BuildStrategy()
        self._graphs = {}

    def with_data_parallel(self, loss_name=None, build_strategy=None, exec_strategy=None, share_vars_from=None,
                           places=None):
        """data parallelism over the job's ranks (reference compiler.py:178). One process drives
        one MI355X: with more than one rank (``torch.distributed`` initialised — RCCL / gloo) every
        gradient of the program's optimizer ops is all-reduced (mean) in buckets whose collectives
        start right after their last gradient op and are waited for before the update (the static
        fleet DP pass). Several places in one process are refused: start one process per GPU."""
        if build_strategy is not None:
            self._build_strategy = build_strategy
        if places is not None and len(list(places)) > 1:
            raise ValueError("with_data_parallel: one process per GPU on MI355X — start one process per device "
                             "(paddle.distributed.launch / spawn) instead of passing several places")
        import torch.distributed as tdist
        env_world = int(os.environ.get("PADDLE_TRAINERS_NUM", "1"))
        if tdist.is_available() and tdist.is_initialized():
            world = tdist.get_world_size()
        elif env_world > 1:
            raise RuntimeError(f"with_data_parallel: PADDLE_TRAINERS_NUM={env_world} but no process group is "
                               "initialised; call paddle.distributed.init_parallel_env() (or fleet.init) first")
        else:
            world = 1
        if world > 1:
            mb = getattr(self._build_strategy, "fuse_grad_size_in_MB", None) or 64
            data_parallel_program(self._program, world, int(mb * 1024 * 1024))
        self._dp_world = world
        return self

    def _run(self, feed, fetch_list, scope=None):
        has_opt = any(is_train_op(op) for op in self._program.global_block().ops)
        if not self._build_strategy.use_hip_graph or has_opt or not torch.cuda.is_available() \
                or has_control_flow(self._program) or (scope is not None and scope is not _global_scope):
            return run_program(self._program, feed, fetch_list, scope)   # (branches cannot be captured)
        key = tuple((k, tuple(np.shape(v if not isinstance(v, Tensor) else v._t)), str(getattr(v, "dtype", "")))
                    for k, v in sorted(feed.items()))
        ent = self._graphs.get(key)
        if ent is None:
            static_in = {k: _wrap((v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))).to(_core.default_device()).clone())
                         for k, v in feed.items()}
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s), torch.no_grad():
                for _ in range(2):
                    run_program(self._program, static_in, fetch_list)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(g):
                outs = run_program(self._program, static_in, fetch_list)
            ent = (g, static_in, outs)
            self._graphs[key] = ent
        g, static_in, outs = ent
        for k, v in feed.items():
            src = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
            static_in[k]._t.copy_(src)
        g.replay()
        return outs


# ----------------------------------------------------------------------------- serialisation
def prune_ops(ops, fetch_vars):
    """Keep only the ops the fetch targets depend on (reference: Program._prune)."""
    if not fetch_vars:
        return list(ops)
    needed = {id(v) for v in fetch_vars}
    kept = []
    for op in reversed(ops):
        if any(id(v) in needed for v in _iter_vars(op.outputs)):
            kept.append(op)
            needed.update(id(v) for v in _iter_vars((op.args, op.kwargs)))
            needed.update(id(v) for v in _iter_vars(op.attrs.get("captured", [])))
    return kept[::-1]


def _resolve_fn(qual):
    fn = OP_REGISTRY.get(qual)
    if fn is not None:
        return fn
    import importlib
    mod, _, name = qual.rpartition(".")
    m = importlib.import_module(mod)
    f = getattr(m, name)
    return getattr(f, "__wrapped_op__", f)
