"""``paddle.fluid.io`` (reference: python/paddle/fluid/io.py): 1.x persistence.

* ``save_vars`` / ``save_params`` / ``save_persistables``: one LoDTensor stream file per variable
  under ``dirname`` (the ``save`` op's format), or every variable in ``filename`` as one
  ``save_combine`` stream sorted by name; the ``load_*`` functions read either layout.
* ``save_inference_model`` writes ``dirname/__model__`` (or ``model_filename``) as a
  framework.proto ProgramDesc plus the parameters in the same two layouts;
  ``load_inference_model`` returns ``[program, feed_names, fetch_targets]``.
* ``save`` / ``load`` / ``load_program_state`` / ``set_program_state`` are the 2.x static ones.
"""
from __future__ import annotations

import os

from ..framework.core import Tensor, Parameter
from ..static import (save, load, load_program_state, set_program_state, serialize_program,  # noqa: F401
                      deserialize_program, deserialize_persistables)
from ..static.program import default_main_program, Program
from ..static import proto as pb
from ..io import DataLoader  # noqa: F401
from .reader import PyReader  # noqa: F401

__all__ = ["save_vars", "save_params", "save_persistables", "load_vars", "load_params", "load_persistables",
           "save_inference_model", "load_inference_model", "batch", "save", "load", "load_program_state",
           "set_program_state", "get_program_parameter", "get_program_persistable_vars", "PyReader", "DataLoader"]


def is_parameter(var):
    return isinstance(var, Parameter)


def is_persistable(var):
    return bool(getattr(var, "persistable", False)) or isinstance(var, Parameter)


def get_program_parameter(program):
    return list(program.all_parameters())


def get_program_persistable_vars(program):
    seen, out = set(), []
    for v in list(program.all_parameters()) + [v for v in program.list_vars() if is_persistable(v)]:
        if id(v) not in seen:
            seen.add(id(v))
            out.append(v)
    return out


def _select(main_program, vars, predicate):
    prog = main_program or default_main_program()
    if vars is not None:
        return list(vars)
    return [v for v in get_program_persistable_vars(prog) if predicate(v)]


def _value(v):
    return v._t if isinstance(v, Tensor) else v


def save_vars(executor, dirname, main_program=None, vars=None, predicate=None, filename=None):
    vs = _select(main_program, vars, predicate or is_persistable)
    os.makedirs(dirname, exist_ok=True)
    if filename is None:
        for v in vs:
            with open(os.path.join(dirname, v.name), "wb") as f:
                f.write(pb.tensor_to_stream(_value(v).detach().cpu()))
        return
    with open(os.path.join(dirname, filename), "wb") as f:
        for v in sorted(vs, key=lambda v: v.name):
            f.write(pb.tensor_to_stream(_value(v).detach().cpu()))


def save_params(executor, dirname, main_program=None, filename=None):
    return save_vars(executor, dirname, main_program, None, is_parameter, filename)


def save_persistables(executor, dirname, main_program=None, filename=None):
    return save_vars(executor, dirname, main_program, None, is_persistable, filename)


def _assign(v, t):
    if isinstance(v, Tensor):
        v.set_value(t.to(v._t.dtype).cpu().numpy()) if t.dtype != v._t.dtype else v.set_value(t.cpu().numpy())


def load_vars(executor, dirname, main_program=None, vars=None, predicate=None, filename=None):
    vs = _select(main_program, vars, predicate or is_persistable)
    if filename is None:
        for v in vs:
            path = os.path.join(dirname, v.name)
            if not os.path.exists(path):
                raise ValueError(f"no saved value for variable {v.name!r} in {dirname}")
            with open(path, "rb") as f:
                t, _, _ = pb.tensor_from_stream(f.read(), 0)
            _assign(v, t)
        return
    with open(os.path.join(dirname, filename), "rb") as f:
        data = f.read()
    off = 0
    for v in sorted(vs, key=lambda v: v.name):
        t, _, off = pb.tensor_from_stream(data, off)
        _assign(v, t)


def load_params(executor, dirname, main_program=None, filename=None):
    return load_vars(executor, dirname, main_program, None, is_parameter, filename)


def load_persistables(executor, dirname, main_program=None, filename=None):
    return load_vars(executor, dirname, main_program, None, is_persistable, filename)


def save_inference_model(dirname, feeded_var_names, target_vars, executor, main_program=None, model_filename=None,
                         params_filename=None, export_for_deployment=True, program_only=False, clip_extra=False):
    from ..static.serialize import program_to_desc
    prog = (main_program or default_main_program()).clone(for_test=True)
    blk = prog.global_block()
    names = [feeded_var_names] if isinstance(feeded_var_names, str) else list(feeded_var_names)
    feeds = [blk.vars[n] for n in names]
    targets = list(target_vars) if isinstance(target_vars, (list, tuple)) else [target_vars]
    os.makedirs(dirname, exist_ok=True)
    desc, persist = program_to_desc(prog, feeds, targets)
    with open(os.path.join(dirname, model_filename or "__model__"), "wb") as f:
        f.write(desc.SerializeToString())
    if program_only:
        return [v.name for v in targets]
    if params_filename is None:
        for n, v in persist.items():
            with open(os.path.join(dirname, n), "wb") as f:
                f.write(pb.tensor_to_stream(_value(v).detach().cpu()))
    else:
        with open(os.path.join(dirname, params_filename), "wb") as f:
            for n in sorted(persist):
                f.write(pb.tensor_to_stream(_value(persist[n]).detach().cpu()))
    return [v.name for v in targets]


def load_inference_model(dirname, executor, model_filename=None, params_filename=None, pserver_endpoints=None):
    from ..static.serialize import parse_program, persistable_names, load_persistables as _lp
    with open(os.path.join(dirname, model_filename or "__model__"), "rb") as f:
        stub = deserialize_program(f.read())
    if params_filename is not None:
        with open(os.path.join(dirname, params_filename), "rb") as f:
            data = f.read()
    else:
        data = b""
        for n in persistable_names(stub.desc):
            with open(os.path.join(dirname, n), "rb") as f:
                data += f.read()
    _ = (parse_program, _lp)
    prog = deserialize_persistables(stub, data, executor)
    return [prog, [v.name for v in stub.feeds], stub.fetches]


def batch(reader, batch_size, drop_last=False):
    from ..reader import batch as _batch
    return _batch(reader, batch_size, drop_last)


_ = Program
