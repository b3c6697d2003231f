"""``paddle.device.cuda.graphs`` on hipGraph (reference: python/paddle/device/cuda/graphs.py:38-118,
paddle/fluid/platform/cuda_graph_with_memory_pool.cc).

The reference records the kernels of a dygraph region (``CUDAGraph.capture_begin`` /
``capture_end`` / ``replay``) or of a to_static function (``wrap_cuda_graph``) into a CUDA graph
with its own memory pool. On MI355X the same object is a hipGraph (``torch.cuda.CUDAGraph`` is
hipGraph on ROCm): every HIP kernel of this framework launches on the current stream, so a whole
training step — forward, backward and the fused optimizer kernels, ~700 launches for ResNet-50 —
replays as ONE graph launch and the host's per-op dispatch cost leaves the step.

What a replay does and does not do (same contract as the reference's CUDA graphs):
  * it re-runs the captured device work on the captured buffers: inputs must be copied into the
    tensors the capture read (``wrap_cuda_graph`` does that), outputs land in the same tensors
    every time;
  * host-side values read during the capture are frozen into the graph (a Python-float learning
    rate, an optimizer step counter used on the host): schedule them on the device or recapture;
  * no host synchronisation may happen inside the captured region (``.item()``, ``.numpy()``).

Capture modes map to ``hipStreamCaptureMode``: ``global`` / ``thread_local`` / ``relaxed``.
Memory pools: ``"default"`` gives each graph a private pool, ``"new"`` a fresh shared handle,
and passing a wrapped function or Layer shares that graph's pool (reference ``memory_pool``).
"""
from __future__ import annotations

import gc
import os

import torch

__all__ = ["CUDAGraph", "wrap_cuda_graph", "is_cuda_graph_supported"]

ALL_MODES = ["global", "thread_local", "relaxed"]
_NO_DEBUG = os.environ.get("PHA_GRAPH_DEBUG", "1") == "0"


def is_cuda_graph_supported():
    """hipGraph capture needs a visible GPU"""
    return torch.cuda.is_available()


class CUDAGraph:
    """One captured hipGraph. ``capture_begin`` moves the calling thread onto a private side
    stream (graph capture cannot run on the legacy default stream) that waits for the current
    stream; ``capture_end`` instantiates the graph and joins the side stream back."""

    _next_id = 0

    def __init__(self, place=None, mode="thread_local", pool=None, _stream=None):
        if mode not in ALL_MODES:
            raise ValueError(f"mode must be one of {ALL_MODES}, got {mode!r}")
        if not is_cuda_graph_supported():
            raise RuntimeError("CUDAGraph needs a HIP device (no GPU visible)")
        dev = None
        if place is not None:
            dev = place.get_device_id() if hasattr(place, "get_device_id") else int(place)
        self._device = torch.cuda.current_device() if dev is None else dev
        self._mode = mode
        self._pool = pool
        self._graph = None
        self._stream = None
        self._fixed_stream = _stream   # captures that must share one stream (forward + backward)
        self._no_debug = False
        self._stream_ctx = None
        self._prev_stream = None
        self.id = CUDAGraph._next_id
        CUDAGraph._next_id += 1

    def capture_begin(self):
        if self._graph is not None:
            raise RuntimeError("graph already captured; call reset() before capturing again")
        torch.cuda.synchronize(self._device)
        gc.collect()
        self._graph = torch.cuda.CUDAGraph()
        if not _NO_DEBUG and not self._no_debug:
            self._graph.enable_debug_mode()   # keeps the graph template for print_to_dot_files
        self._prev_stream = torch.cuda.current_stream(self._device)
        self._stream = self._fixed_stream or torch.cuda.Stream(device=self._device)
        self._stream.wait_stream(self._prev_stream)
        self._stream_ctx = torch.cuda.stream(self._stream)
        self._stream_ctx.__enter__()
        try:
            self._graph.capture_begin(pool=self._pool, capture_error_mode=self._mode)
        except Exception:
            self._stream_ctx.__exit__(None, None, None)
            self._stream_ctx = None
            self._graph = None
            raise

    def capture_end(self):
        if self._stream_ctx is None:
            raise RuntimeError("capture_end() without capture_begin()")
        try:
            self._graph.capture_end()
        finally:
            self._stream_ctx.__exit__(None, None, None)
            self._stream_ctx = None
            self._prev_stream.wait_stream(self._stream)

    def replay(self):
        if self._graph is None or self._stream_ctx is not None:
            raise RuntimeError("replay() needs a finished capture")
        self._graph.replay()

    def reset(self):
        if self._graph is not None:
            self._graph.reset()
        self._graph = None

    def pool(self):
        """memory-pool handle of this graph (share it with another capture)"""
        return self._graph.pool() if self._graph is not None else self._pool

    def print_to_dot_files(self, dirname, flags=None):
        """write the captured graph as Graphviz ``.dot`` (hipGraphDebugDotPrint); ``flags`` is
        accepted for parity — the HIP runtime prints its full description"""
        if self._graph is None:
            raise RuntimeError("nothing captured")
        if not isinstance(dirname, (str, bytes)):
            dirname = dirname.name
        os.makedirs(dirname, exist_ok=True)
        path = os.path.join(dirname, f"graph_{self.id}.dot")
        self._graph.debug_dump(path)
        return path


def _tensors_of(obj, out):
    from ...framework.core import Tensor
    if isinstance(obj, Tensor):
        out.append(obj._t)
    elif isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _tensors_of(o, out)
    elif isinstance(obj, dict):
        for k in sorted(obj):
            _tensors_of(obj[k], out)
    return out


def _signature(obj):
    """hashable description of the non-tensor structure of the arguments (shape / dtype of
    tensors, value of everything else): a different signature gets its own graph"""
    from ...framework.core import Tensor
    if isinstance(obj, Tensor):
        obj = obj._t
    if isinstance(obj, torch.Tensor):
        return ("T", tuple(obj.shape), str(obj.dtype), str(obj.device))
    if isinstance(obj, (list, tuple)):
        return (type(obj).__name__,) + tuple(_signature(o) for o in obj)
    if isinstance(obj, dict):
        return ("dict",) + tuple((k, _signature(obj[k])) for k in sorted(obj))
    return ("V", repr(obj))


def _detach_any(obj):
    from ...framework.core import Tensor, _wrap
    if isinstance(obj, Tensor):
        return _wrap(obj._t.detach())
    if isinstance(obj, torch.Tensor):
        return obj.detach()
    if isinstance(obj, (list, tuple)):
        return type(obj)(_detach_any(o) for o in obj)
    if isinstance(obj, dict):
        return {k: _detach_any(v) for k, v in obj.items()}
    return obj


def _rebuild(obj, it):
    """``obj`` with every tensor replaced by the next one of ``it`` (wrapped like the original)"""
    from ...framework.core import Tensor, _wrap
    if isinstance(obj, Tensor):
        return _wrap(next(it))
    if isinstance(obj, torch.Tensor):
        return next(it)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_rebuild(o, it) for o in obj)
    if isinstance(obj, dict):
        return {k: _rebuild(obj[k], it) for k in sorted(obj)}
    return obj


class _AutogradGraphs:
    """Forward and backward of a differentiable call, each captured once as a hipGraph — the
    reference's ``run_program`` op keeps a forward and a backward program for a wrapped Layer
    (python/paddle/fluid/dygraph/dygraph_to_static/partial_program.py). Every call replays the
    forward through an autograd Function whose backward replays the captured backward, so the
    eager tape around it (``loss.backward()`` of the caller, gradient accumulation into the
    Layer's parameters) works like an un-graphed call."""

    def __init__(self, fn, args, kwargs, params, mode, pool):
        ins = _tensors_of((args, kwargs), [])
        self.static_in = [t.detach().clone().requires_grad_(t.requires_grad) for t in ins]
        # a wrapped Layer's parameters (framework Parameters, whose torch tensor is ``_t``): during
        # warmup and capture the Layer runs on fresh leaf aliases of the same storage. The real
        # leaves' AccumulateGrad nodes were made by eager calls on another stream and may still be
        # referenced by the caller's last autograd graph; routing the captured backward through them
        # makes autograd join the capture with that stream (an invalid capture: the HIP runtime
        # crashed at instantiation). Replays read the parameters' live storage; _GraphedCall hands
        # the captured gradients to the real leaves.
        owners = [p for p in params if getattr(p, "_t", p).requires_grad]
        self.params = [getattr(p, "_t", p) for p in owners]
        aliases = [t.detach().requires_grad_(True) for t in self.params]
        swap = [o for o in owners if hasattr(o, "_t")]
        for o, a in zip(owners, aliases):
            if hasattr(o, "_t"):
                o._t = a
        try:
            self._capture(fn, args, kwargs, aliases if swap else self.params, mode, pool)
        finally:
            for o, t in zip(owners, self.params):
                if hasattr(o, "_t"):
                    o._t = t

    def _capture(self, fn, args, kwargs, params, mode, pool):
        sargs, skw = _rebuild((args, kwargs), iter(self.static_in))
        diff = [t for t in self.static_in if t.requires_grad] + list(params)
        stream = torch.cuda.Stream()
        stream.wait_stream(torch.cuda.current_stream())
        # warm the autograd path on the capture stream (lazy init, allocator growth)
        with torch.cuda.stream(stream):
            outs = _tensors_of(fn(*sargs, **skw), [])
            req = [o for o in outs if o.requires_grad]
            if req:
                torch.autograd.grad(req, diff, [torch.ones_like(o) for o in req], allow_unused=True)
            del outs, req
        torch.cuda.current_stream().wait_stream(stream)
        self.fwd = CUDAGraph(mode=mode, pool=pool, _stream=stream)
        self.fwd.capture_begin()
        try:
            out_obj = fn(*sargs, **skw)
        finally:
            self.fwd.capture_end()
        self.out_obj = out_obj
        self.static_out = _tensors_of(out_obj, [])
        self.out_req = [o.requires_grad for o in self.static_out]
        self.static_gout = [torch.empty_like(o) for o, r in zip(self.static_out, self.out_req) if r]
        self.bwd = CUDAGraph(mode=mode, pool=self.fwd.pool(), _stream=stream)
        self.bwd.capture_begin()
        try:
            grads = torch.autograd.grad([o for o, r in zip(self.static_out, self.out_req) if r], diff,
                                        self.static_gout, allow_unused=True)
        finally:
            self.bwd.capture_end()
        self.static_grad = list(grads)
        self.in_req = [t.requires_grad for t in self.static_in]
        self.generation = 0   # forward replays so far: the saved activations belong to the latest

    def __call__(self, args, kwargs):
        ins = _tensors_of((args, kwargs), [])
        outs = _GraphedCall.apply(self, len(ins), *ins, *self.params)
        return _rebuild(self.out_obj, iter(outs))


class _GraphedCall(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g, n_in, *tensors):
        for dst, src in zip(g.static_in, tensors[:n_in]):
            if dst.data_ptr() != src.data_ptr():
                dst.detach().copy_(src)
        g.fwd.replay()
        g.generation += 1
        ctx.g, ctx.n_in, ctx.generation = g, n_in, g.generation
        outs = tuple(o.detach() for o in g.static_out)
        ctx.mark_non_differentiable(*[o for o, r in zip(outs, g.out_req) if not r])
        return outs

    @staticmethod
    def backward(ctx, *gouts):
        g = ctx.g
        if ctx.generation != g.generation:
            # the captured backward reads the static activations of the LATEST forward replay; an
            # older call's gradients would silently come from the newer call's activations
            raise RuntimeError(
                "wrap_cuda_graph: backward of a graphed call after a newer forward replay of the same "
                "graph (the static activation buffers were overwritten). Run backward before calling "
                "the graphed Layer again, or wrap each call site (weight sharing, several micro-batches "
                "per backward) in its own wrap_cuda_graph")
        k = 0
        for go, r in zip(gouts, g.out_req):
            if r:
                if go is None:
                    g.static_gout[k].zero_()
                else:
                    g.static_gout[k].copy_(go)
                k += 1
        g.bwd.replay()
        grads, k = [], 0
        for r in g.in_req:
            if r:
                gr = g.static_grad[k]
                grads.append(None if gr is None else gr.clone())
                k += 1
            else:
                grads.append(None)
        for gr in g.static_grad[k:]:
            grads.append(None if gr is None else gr.clone())
        return (None, None) + tuple(grads)


class GraphedFunction:
    """``wrap_cuda_graph`` result in dygraph mode. Call 1..warmup: eager, on a side stream (lazy
    initialisation, per-shape GEMM picks and allocator growth happen outside the capture).

    * A differentiable call (grad enabled and an input or, for a wrapped Layer, a parameter
      requires grad) captures the forward and the backward as two hipGraphs
      (:class:`_AutogradGraphs`): the caller backpropagates through the result as through an eager
      call and the parameters accumulate their gradients.
    * Anything else — e.g. a whole training step that calls ``backward()`` and the optimizer
      itself — is captured as one graph: the next call captures and then replays once, so every
      call performs the work exactly once; later calls copy the tensor arguments into the
      captured inputs and replay.

    Outputs are the captured tensors (overwritten by the next call), as in the reference."""

    def __init__(self, function, mode="thread_local", memory_pool="default", warmup=1, params=None):
        self._params = params   # a wrapped Layer's parameters (torch tensors), called lazily
        if mode not in ALL_MODES:
            raise ValueError(f"mode must be one of {ALL_MODES}, got {mode!r}")
        self._fn = function
        self._mode = mode
        self._warmup = warmup
        if memory_pool == "default":
            self._pool = None
        elif memory_pool == "new":
            self._pool = torch.cuda.graph_pool_handle() if is_cuda_graph_supported() else None
        elif isinstance(memory_pool, GraphedFunction):
            self._pool = memory_pool._pool if memory_pool._pool is not None else memory_pool._first_pool()
        elif hasattr(memory_pool, "_cuda_graph") and isinstance(memory_pool._cuda_graph, GraphedFunction):
            self._pool = memory_pool._cuda_graph._first_pool()
        else:
            raise ValueError("memory_pool must be 'default', 'new', or a wrapped function / Layer")
        self._entries = {}
        self._calls = {}

    def _first_pool(self):
        for ent in self._entries.values():
            return ent.fwd.pool() if isinstance(ent, _AutogradGraphs) else ent[0].pool()
        return None

    def _side_stream(self):
        if getattr(self, "_stream", None) is None:
            self._stream = torch.cuda.Stream()
        return self._stream

    def _differentiable(self, args, kwargs):
        if not torch.is_grad_enabled():
            return False
        if any(t.requires_grad for t in _tensors_of((args, kwargs), [])):
            return True
        return self._params is not None and any(getattr(p, "_t", p).requires_grad for p in self._params())

    def __call__(self, *args, **kwargs):
        if not is_cuda_graph_supported():
            return self._fn(*args, **kwargs)
        diff = self._differentiable(args, kwargs)
        key = (diff, _signature((args, kwargs)))
        ent = self._entries.get(key)
        if diff:
            if ent is None:
                n = self._calls.get(key, 0)
                self._calls[key] = n + 1
                if n < self._warmup:
                    return self._fn(*args, **kwargs)
                ent = _AutogradGraphs(self._fn, args, kwargs, self._params() if self._params else [], self._mode,
                                      self._pool)
                self._entries[key] = ent
            return ent(args, kwargs)
        if ent is None:
            n = self._calls.get(key, 0)
            self._calls[key] = n + 1
            if n < self._warmup:
                # on the stream the capture will use, and the result detached: the warmup's
                # autograd graph (its AccumulateGrad nodes) must be gone before the capture, or
                # autograd syncs the capture against the stale nodes' stream
                s = self._side_stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    out = self._fn(*args, **kwargs)
                torch.cuda.current_stream().wait_stream(s)
                return _detach_any(out)
            g = CUDAGraph(mode=self._mode, pool=self._pool, _stream=self._side_stream())
            g.capture_begin()
            try:
                out = self._fn(*args, **kwargs)
            finally:
                g.capture_end()
            ent = (g, _tensors_of((args, kwargs), []), out)
            self._entries[key] = ent
            g.replay()   # the capture itself ran nothing
            return out
        g, static_in, out = ent
        for dst, src in zip(static_in, _tensors_of((args, kwargs), [])):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
        g.replay()
        return out

    def reset(self):
        for ent in self._entries.values():
            if isinstance(ent, _AutogradGraphs):
                ent.fwd.reset()
                ent.bwd.reset()
            else:
                ent[0].reset()
        self._entries.clear()
        self._calls.clear()


def wrap_cuda_graph(function, mode="thread_local", memory_pool="default", warmup=1):
    """Reference ``wrap_cuda_graph``. Dygraph: a :class:`GraphedFunction` around ``function``
    (a Layer's forward is wrapped in place and the Layer returned). Static mode: the ops the
    function records are tagged ``_cuda_graph_attr`` = "mode;pool;id" like the reference's
    ``_cuda_graph_guard`` (carried in the Program IR; ``CompiledProgram`` with
    ``build_strategy.use_hip_graph`` replays a program as one hipGraph).

    Limitation of a differentiable graphed call: its outputs and saved activations are the
    captured static buffers, so only the LATEST call can be backpropagated. Calling the graphed
    Layer twice before backward (a weight-shared block, several micro-batches, several losses)
    makes the older call's backward raise instead of silently using the newer activations."""
    from ...framework import core as _core
    from ...nn import Layer
    if mode not in ALL_MODES:
        raise ValueError(f"mode must be one of {ALL_MODES}, got {mode!r}")
    if not _core.in_dynamic_mode():
        return _static_guard(function, mode, memory_pool)
    if isinstance(function, Layer):
        layer = function
        gf = GraphedFunction(layer.forward, mode, memory_pool, warmup, params=lambda: list(layer.parameters()))
        layer._cuda_graph = gf
        layer.forward = gf
        return layer
    return GraphedFunction(function, mode, memory_pool, warmup)


_static_ids = [0]


def _static_guard(function, mode, memory_pool):
    if memory_pool not in ("default", "new"):
        raise ValueError("memory_pool should be 'default' or 'new' under static mode")
    gid = _static_ids[0]
    _static_ids[0] += 1
    attr = f"{mode};{0 if memory_pool == 'default' else gid + 1};{gid}"

    def run(*args, **kwargs):
        from ...static import default_main_program
        block = default_main_program().global_block()
        n0 = len(block.ops)
        out = function(*args, **kwargs)
        for op in block.ops[n0:]:
            op.attrs["_cuda_graph_attr"] = attr
        return out
    return run
