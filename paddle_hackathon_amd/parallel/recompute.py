"""Activation recompute (reference: python/paddle/distributed/fleet/utils/recompute.py).

Forward runs under no_grad and keeps only the inputs; backward re-runs the
function with the saved RNG state (CPU + HIP generators, and the TP RNG tracker)
so dropout masks match, then back-propagates through the recomputed graph.
"""
from __future__ import annotations

import threading

import torch

from ..framework.core import Tensor, _wrap

__all__ = ["recompute", "recompute_sequential"]


class _Nesting(threading.local):
    def __init__(self):
        self.depth = 0
        self.deferred = []


_NEST = _Nesting()


def queue_outer_callback(cb):
    """queue ``cb`` to run when the OUTERMOST backward in progress finishes. Gradient hooks firing
    inside a recomputed segment run in the nested backward of _Recompute.backward, and
    ``queue_callback`` would attach to that nested graph task — a reducer / sharding finaliser
    would then run after the first recomputed segment and miss every later gradient. Inside a
    recompute backward the callback is held and queued on the outer task when the segment ends."""
    if _NEST.depth > 0:
        if cb not in _NEST.deferred:
            _NEST.deferred.append(cb)
    else:
        torch.autograd.Variable._execution_engine.queue_callback(cb)


def _tracker_states():
    from .mp_layers import get_rng_state_tracker
    return get_rng_state_tracker().get_states_tracker()


class _Recompute(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fn, preserve_rng, kwargs, n_tensors, *args):
        ctx.fn, ctx.preserve, ctx.kwargs = fn, preserve_rng, kwargs
        ctx.kinds = [isinstance(a, torch.Tensor) for a in args]
        ctx.nontensors = [a for a in args if not isinstance(a, torch.Tensor)]
        if preserve_rng:
            ctx.cpu_state = torch.get_rng_state()
            ctx.cuda_state = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
            ctx.tracker = _tracker_states()
        ctx.save_for_backward(*[a for a in args if isinstance(a, torch.Tensor)])
        with torch.no_grad():
            out = fn(*[_wrap(a) if isinstance(a, torch.Tensor) else a for a in args], **kwargs)
        if isinstance(out, (tuple, list)):
            ctx.multi = True
            return tuple(o._t if isinstance(o, Tensor) else o for o in out)
        ctx.multi = False
        return out._t

    @staticmethod
    def backward(ctx, *grads):
        tens = list(ctx.saved_tensors)
        it_t, it_n = iter(tens), iter(ctx.nontensors)
        inputs = []
        for k in ctx.kinds:
            if k:
                t = next(it_t).detach()
                t.requires_grad_(True)
                inputs.append(t)
            else:
                inputs.append(next(it_n))
        if ctx.preserve:
            from .mp_layers import get_rng_state_tracker
            cur_cpu = torch.get_rng_state()
            cur_cuda = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
            cur_tr = _tracker_states()
            torch.set_rng_state(ctx.cpu_state)
            if ctx.cuda_state is not None:
                torch.cuda.set_rng_state(ctx.cuda_state)
            get_rng_state_tracker().set_states_tracker(ctx.tracker)
        try:
            with torch.enable_grad():
                out = ctx.fn(*[_wrap(a) if isinstance(a, torch.Tensor) else a for a in inputs], **ctx.kwargs)
        finally:
            if ctx.preserve:
                torch.set_rng_state(cur_cpu)
                if cur_cuda is not None:
                    torch.cuda.set_rng_state(cur_cuda)
                get_rng_state_tracker().set_states_tracker(cur_tr)
        outs = out if isinstance(out, (tuple, list)) else (out,)
        outs_t = [o._t if isinstance(o, Tensor) else o for o in outs]
        pairs = [(o, g) for o, g in zip(outs_t, grads) if isinstance(o, torch.Tensor) and o.requires_grad and g is not None]
        if pairs:
            _NEST.depth += 1
            try:
                torch.autograd.backward([p[0] for p in pairs], [p[1] for p in pairs])
            finally:
                _NEST.depth -= 1
            if _NEST.depth == 0 and _NEST.deferred:
                cbs, _NEST.deferred = _NEST.deferred, []
                for cb in cbs:   # this node runs in the outer backward: its graph task takes them
                    torch.autograd.Variable._execution_engine.queue_callback(cb)
        gin = [t.grad if isinstance(t, torch.Tensor) else None for t in inputs]
        return (None, None, None, None, *gin)


def recompute(function, *args, **kwargs):
    preserve = kwargs.pop("preserve_rng_state", True)
    kwargs.pop("use_reentrant", None)
    targs = [a._t if isinstance(a, Tensor) else a for a in args]
    out = _Recompute.apply(function, preserve, kwargs, sum(isinstance(a, torch.Tensor) for a in targs), *targs)
    if isinstance(out, tuple):
        return tuple(_wrap(o) if isinstance(o, torch.Tensor) else o for o in out)
    return _wrap(out)


def recompute_sequential(ctx, functions, *args, **kwargs):
    segments = ctx.get("segments", 1)
    funcs = list(functions.children()) if hasattr(functions, "children") else list(functions)
    n = len(funcs)
    per = max(1, (n + segments - 1) // segments)

    def run(start, end):
        def f(x):
            for fn in funcs[start:end]:
                x = fn(x)
            return x
        return f
    x = args[0]
    for s in range(0, n, per):
        x = recompute(run(s, min(n, s + per)), x)
    return x
