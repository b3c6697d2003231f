"""Op dispatch boundary.

Every public op (``paddle.add``, ``F.linear`` …) is wrapped once by
:func:`register_ops`. In dynamic mode the wrapper is a single flag test and a
tail call. In static mode (``paddle.enable_static()``) a call whose arguments
contain static ``Variable`` s is *recorded* into the current ``Program`` block
instead — shapes/dtypes are inferred by running the op on ``meta`` tensors,
the same role phi's InferMeta plays in the reference
(paddle/phi/infermeta/*, python/paddle/fluid/framework.py:Block.append_op).
"""
from __future__ import annotations

import functools

from .core import _mode


def _record_hook(fn, name, args, kwargs):
    from ..static.program import record_op
    return record_op(fn, name, args, kwargs)


def _traced(fn, name, args, kwargs):
    if _mode.trace:
        from ..profiler import _op_range
        with _op_range(name, "Operator"):
            out = fn(*args, **kwargs)
    else:
        out = fn(*args, **kwargs)
    if _mode.check_nan_inf:
        from .nan_inf import check_outputs
        check_outputs(name, out)
    return out


def static_op(fn, name=None):
    opname = name or fn.__name__

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        if _mode.static and _mode.record_depth == 0:
            return _record_hook(fn, opname, args, kwargs)
        if _mode.trace or _mode.check_nan_inf:
            return _traced(fn, opname, args, kwargs)
        return fn(*args, **kwargs)

    wrapper.__wrapped_op__ = fn
    return wrapper


def register_ops(namespace, names):
    """Wrap ``namespace[name]`` for every public op name in place."""
    for n in names:
        f = namespace.get(n)
        if callable(f) and not isinstance(f, type) and not hasattr(f, "__wrapped_op__"):
            namespace[n] = static_op(f, n)
