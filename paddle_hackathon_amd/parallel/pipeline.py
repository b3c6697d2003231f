"""Pipeline parallelism (reference: python/paddle/distributed/fleet/meta_parallel/
{parallel_layers/pp_layers.py, pipeline_parallel.py, pp_utils/p2p_communication.py}).

``PipelineLayer`` builds only this stage's slice of a LayerDesc list (uniform or
"layer:Name" segmentation); ``PipelineParallel.train_batch`` runs the 1F1B schedule
over ``accumulate_steps`` micro-batches. Stage-to-stage activations and gradients
move with batched isend/irecv pairs on the pipe group (RCCL p2p over xGMI on GPU),
combining the "send forward + receive backward" of the steady state in one
batched call so neither direction can block the other.
"""
from __future__ import annotations

import math
import re

import torch
import torch.distributed as dist

from ..framework.core import Tensor, _wrap
from ..nn.layer.layers import Layer
from ..nn.layer.container import LayerList
from . import collective as C

__all__ = ["LayerDesc", "SharedLayerDesc", "PipelineLayer", "PipelineParallel"]


class LayerDesc:
    def __init__(self, layer_func, *inputs, **kwargs):
        self.layer_func, self.inputs, self.kwargs = layer_func, inputs, kwargs
        if not issubclass(layer_func, Layer):
            raise TypeError("LayerDesc expects a Layer subclass")

    def build_layer(self):
        return self.layer_func(*self.inputs, **self.kwargs)

    def __repr__(self):
        return f"LayerDesc({self.layer_func.__name__})"


class SharedLayerDesc(LayerDesc):
    def __init__(self, key, layer_func, forward_func=None, shared_weight_attr="weight", *inputs, **kwargs):
        super().__init__(layer_func, *inputs, **kwargs)
        self.layer_name, self.forward_func, self.shared_weight_attr = key, forward_func, shared_weight_attr


class _SegmentLayers:
    def __init__(self, descs, num_parts, method="uniform"):
        self.descs, self.num_parts, self.method = descs, num_parts, method

    def do_segment(self):
        n = len(self.descs)
        if self.method == "uniform":
            base, extra = divmod(n, self.num_parts)
            bounds = [0]
            for i in range(self.num_parts):
                bounds.append(bounds[-1] + base + (1 if i < extra else 0))
            return bounds
        if self.method.startswith("layer:"):
            name = self.method.split(":", 1)[1]
            pat = re.compile(name, re.IGNORECASE)
            idx = [i for i, d in enumerate(self.descs)
                   if pat.search((d.layer_func.__name__ if isinstance(d, LayerDesc) else type(d).__name__))]
            per, extra = divmod(len(idx), self.num_parts)
            bounds = [0]
            k = 0
            for i in range(1, self.num_parts):
                k += per + (1 if i - 1 < extra else 0)
                bounds.append(idx[k] if k < len(idx) else n)
            bounds.append(n)
            return bounds
        raise ValueError(self.method)


class PipelineLayer(Layer):
    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seg_method="uniform",
                 recompute_interval=0, recompute_ctx=None, num_virtual_pipeline_stages=None):
        super().__init__()
        from . import fleet
        hcg = fleet.fleet._hcg
        if topology is None and hcg is not None:
            topology = hcg.topology()
        self._topo = topology
        if num_stages is None:
            num_stages = topology.get_dim("pipe") if topology is not None else 1
        self._num_stages = num_stages
        self._stage_id = hcg.get_stage_id() if hcg is not None else 0
        self._loss_fn = loss_fn
        self._recompute_interval = recompute_interval
        self._layers_desc = list(layers)
        self.segment_parts = _SegmentLayers(self._layers_desc, num_stages, seg_method).do_segment()
        self._start = self.segment_parts[self._stage_id]
        self._end = self.segment_parts[self._stage_id + 1]
        self.run_function = []
        self.shared_layers = {}
        self.shared_weight_attrs = {}
        self._built = LayerList()
        for i in range(self._start, self._end):
            d = self._layers_desc[i]
            if isinstance(d, SharedLayerDesc):
                if d.layer_name not in self.shared_layers:
                    self.shared_layers[d.layer_name] = d.build_layer()
                    self.shared_weight_attrs[d.layer_name] = d.shared_weight_attr
                layer = self.shared_layers[d.layer_name]
                self._built.append(layer)
                if d.forward_func is not None:
                    ff = d.forward_func
                    self.run_function.append(lambda x, _l=layer, _f=ff: _f(_l, x))
                else:
                    self.run_function.append(layer)
            elif isinstance(d, LayerDesc):
                layer = d.build_layer()
                self._built.append(layer)
                self.run_function.append(layer)
            elif isinstance(d, Layer):
                self._built.append(d)
                self.run_function.append(d)
            else:
                self.run_function.append(d)
        self._shared_groups = self._build_shared_groups(hcg)

    def _build_shared_groups(self, hcg):
        """For every SharedLayerDesc key: the pipe stages using it, one group per pipeline."""
        groups = {}
        keys = {}
        for s in range(self._num_stages):
            for i in range(self.segment_parts[s], self.segment_parts[s + 1]):
                d = self._layers_desc[i]
                if isinstance(d, SharedLayerDesc):
                    keys.setdefault(d.layer_name, set()).add(s)
        if hcg is None or not C.is_initialized():
            return groups
        topo = self._topo
        names = topo.get_hybrid_group_names()
        pipe_axis = names.index("pipe")
        import itertools
        for key in sorted(keys):
            stages = sorted(keys[key])
            if len(stages) < 2:
                continue
            other = [range(topo.get_dim(n)) for n in names if n != "pipe"]
            for coord in itertools.product(*other):
                ranks = []
                for s in stages:
                    c = list(coord)
                    c.insert(pipe_axis, s)
                    ranks.append(topo.get_rank(**dict(zip(names, c))))
                g = C.new_group(ranks)
                if C.get_rank() in ranks:
                    groups[key] = g
        # the norm of a shared weight's (all-reduced, identical) gradient counts on the first
        # stage holding it only (reference: is_firstly_shared in pp_layers.py)
        for key in keys:
            if key in self.shared_layers:
                w = getattr(self.shared_layers[key], self.shared_weight_attrs[key])
                w.is_firstly_shared = self._stage_id == min(keys[key])
        # make shared weights identical (first stage wins)
        for key, g in groups.items():
            if key in self.shared_layers:
                w = getattr(self.shared_layers[key], self.shared_weight_attrs[key])
                dist.broadcast(w._t.data, src=g.ranks[0], group=g.pg)
        return groups

    def shared_parameters(self):
        """the weights tied across stages (SharedLayerDesc): sharding keeps them replicated, so
        their gradients stay whole for the cross-stage all-reduce"""
        return [getattr(self.shared_layers[k], self.shared_weight_attrs[k]) for k in self.shared_layers]

    def allreduce_shared_weight_gradients(self):
        for key, g in self._shared_groups.items():
            if key not in self.shared_layers:
                continue
            w = getattr(self.shared_layers[key], self.shared_weight_attrs[key])
            if w._t.grad is not None:
                dist.all_reduce(w._t.grad, group=g.pg)

    def get_stage_from_index(self, layer_idx):
        for s in range(self._num_stages):
            if self.segment_parts[s] <= layer_idx < self.segment_parts[s + 1]:
                return s
        return self._num_stages - 1

    def forward(self, input):
        x = input
        if self._recompute_interval > 0 and self.training:
            from .recompute import recompute
            fns = self.run_function
            for i in range(0, len(fns), self._recompute_interval):
                chunk = fns[i:i + self._recompute_interval]

                def run(*xs, _c=chunk):
                    y = xs[0] if len(xs) == 1 else xs
                    for f in _c:
                        y = f(y) if not isinstance(y, tuple) else f(*y)
                    return y
                x = recompute(run, *(x if isinstance(x, tuple) else (x,)))
            return x
        for f in self.run_function:
            x = f(*x) if isinstance(x, tuple) else f(x)
        return x


_DT_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.int64: 3, torch.int32: 4, torch.bool: 5, torch.float64: 6}
_CODE_DT = {v: k for k, v in _DT_CODE.items()}


class _P2P:
    """Stage-to-stage transport on the pipe group (batched isend/irecv)."""

    def __init__(self, hcg, device):
        self.hcg = hcg
        self.group = hcg.get_pipe_parallel_group()
        self.pg = self.group.pg
        self.prev = hcg._p2p_prev
        self.next = hcg._p2p_next
        self.device = device
        self.recv_meta = None   # [(shape, dtype)] of activations coming from prev
        self.send_meta_done = False

    def _batch(self, ops):
        if not ops:
            return
        reqs = dist.batch_isend_irecv(ops)
        for r in reqs:
            r.wait()

    def send_meta(self, tensors):
        if self.send_meta_done:
            return
        meta = [len(tensors)]
        for t in tensors:
            meta += [_DT_CODE[t.dtype], t.dim()] + list(t.shape)
        m = torch.tensor([len(meta)] + meta + [0] * (63 - len(meta)), dtype=torch.int64, device=self.device)
        dist.send(m, self.next, group=self.pg)
        self.send_meta_done = True

    def get_meta(self):
        if self.recv_meta is None:
            m = torch.empty(64, dtype=torch.int64, device=self.device)
            dist.recv(m, self.prev, group=self.pg)
            vals = m.tolist()
            n = vals[0]
            meta = vals[1:1 + n]
            cnt = meta[0]
            pos = 1
            out = []
            for _ in range(cnt):
                dt, nd = meta[pos], meta[pos + 1]
                shape = meta[pos + 2:pos + 2 + nd]
                pos += 2 + nd
                out.append((shape, _CODE_DT[dt]))
            self.recv_meta = out
        return self.recv_meta

    def _empty_acts(self):
        return [torch.empty(s, dtype=d, device=self.device) for s, d in self.get_meta()]

    def recv_forward(self):
        bufs = self._empty_acts()
        self._batch([dist.P2POp(dist.irecv, b, self.prev, self.pg) for b in bufs])
        return bufs

    def send_forward(self, outs):
        self.send_meta(outs)
        self._batch([dist.P2POp(dist.isend, o.contiguous(), self.next, self.pg) for o in outs])

    def recv_backward(self, outs):
        bufs = [torch.empty_like(o) for o in outs]
        self._batch([dist.P2POp(dist.irecv, b, self.next, self.pg) for b in bufs])
        return bufs

    def send_backward(self, grads):
        self._batch([dist.P2POp(dist.isend, g.contiguous(), self.prev, self.pg) for g in grads])

    def send_forward_recv_backward(self, outs):
        self.send_meta(outs)
        bufs = [torch.empty_like(o) for o in outs]
        ops = [dist.P2POp(dist.isend, o.contiguous(), self.next, self.pg) for o in outs]
        ops += [dist.P2POp(dist.irecv, b, self.next, self.pg) for b in bufs]
        self._batch(ops)
        return bufs

    def send_backward_recv_forward(self, grads):
        bufs = self._empty_acts()
        ops = [dist.P2POp(dist.isend, g.contiguous(), self.prev, self.pg) for g in grads]
        ops += [dist.P2POp(dist.irecv, b, self.prev, self.pg) for b in bufs]
        self._batch(ops)
        return bufs


def _as_list(x):
    if isinstance(x, (tuple, list)):
        return [v._t if isinstance(v, Tensor) else v for v in x]
    return [x._t if isinstance(x, Tensor) else x]


class PipelineParallel(Layer):
    def __init__(self, layers, hcg, strategy):
        super().__init__()
        if not isinstance(layers, PipelineLayer):
            raise TypeError("PipelineParallel expects a PipelineLayer")
        self._layers = layers
        self._hcg = hcg
        self._strategy = strategy
        cfg = strategy.pipeline_configs if strategy is not None else {"micro_batch_size": 1, "accumulate_steps": 1}
        self.micro_batch_size = cfg["micro_batch_size"]
        self.accumulate_steps = cfg["accumulate_steps"]
        self.num_stages = hcg.get_pipe_parallel_world_size()
        self.stage_id = hcg.get_stage_id()
        self.is_first = self.stage_id == 0
        self.is_last = self.stage_id == self.num_stages - 1
        self._p2p = None
        self._dp_group = hcg.get_data_parallel_group()
        self.total_loss = None

    def _device(self):
        from ..framework.core import default_device
        return default_device()

    def _micro(self, data, i):
        def sl(x):
            if x is None:
                return None
            if isinstance(x, (tuple, list)):
                return type(x)(sl(v) for v in x)
            t = x._t if isinstance(x, Tensor) else x
            b = self.micro_batch_size
            return _wrap(t[i * b:(i + 1) * b])
        return sl(data)

    def _forward_step(self, inputs, labels):
        out = self._layers(inputs)
        if self.is_last:
            loss = self._layers._loss_fn(out, labels) if self._layers._loss_fn is not None else out
            loss = _wrap(loss._t / self.accumulate_steps)
            with torch.no_grad():
                self.total_loss = loss._t.detach().clone() if self.total_loss is None else self.total_loss + loss._t.detach()
            return loss
        return out

    def forward_backward_pipeline(self, data, scaler=None):
        if self._p2p is None:
            self._p2p = _P2P(self._hcg, self._device())
        p2p = self._p2p
        inputs, labels = data if isinstance(data, (tuple, list)) and len(data) == 2 else (data, None)
        n = self.accumulate_steps
        warm = min(self.num_stages - self.stage_id - 1, n)
        steady = n - warm
        in_q, out_q = [], []
        self.total_loss = None
        mb = [0]

        def fwd(recv):
            i = mb[0]
            mb[0] += 1
            if self.is_first:
                x = self._micro(inputs, i)
                x_in = None
            else:
                ts = [t.requires_grad_(t.is_floating_point()) for t in recv]
                x = _wrap(ts[0]) if len(ts) == 1 else tuple(_wrap(t) for t in ts)
                x_in = ts
            out = self._forward_step(x, self._micro(labels, i) if self.is_last else None)
            in_q.append(x_in)
            out_q.append(out)
            return out

        def bwd(grads):
            x_in = in_q.pop(0)
            out = out_q.pop(0)
            if self.is_last:
                loss = out._t
                if scaler is not None:
                    loss = loss * scaler._scale
                torch.autograd.backward(loss)
            else:
                outs = _as_list(out)
                pairs = [(o, g) for o, g in zip(outs, grads) if o.requires_grad]
                torch.autograd.backward([p[0] for p in pairs], [p[1] for p in pairs])
            if x_in is None:
                return None
            return [t.grad if t.grad is not None else torch.zeros_like(t) for t in x_in]

        for _ in range(warm):
            recv = None if self.is_first else p2p.recv_forward()
            out = fwd(recv)
            if not self.is_last:
                p2p.send_forward(_as_list(out))
        recv = None
        if steady > 0 and not self.is_first:
            recv = p2p.recv_forward()
        for i in range(steady):
            last = i == steady - 1
            out = fwd(recv)
            if self.is_last:
                grads = None
            else:
                grads = p2p.send_forward_recv_backward([o.detach() for o in _as_list(out)])
            dx = bwd(grads)
            if last:
                recv = None
                if not self.is_first:
                    p2p.send_backward(dx)
            else:
                if self.is_first:
                    recv = None
                else:
                    recv = p2p.send_backward_recv_forward(dx)
        for _ in range(warm):
            grads = None if self.is_last else p2p.recv_backward(_as_list(out_q[0]))
            dx = bwd(grads)
            if not self.is_first:
                p2p.send_backward(dx)
        self._layers.allreduce_shared_weight_gradients()
        return self._broadcast_loss()

    def _broadcast_loss(self):
        dev = self._device()
        loss = self.total_loss if self.is_last else torch.zeros((), dtype=torch.float32, device=dev)
        loss = loss.float().reshape(()).clone()
        if self.num_stages > 1:
            g = self._hcg.get_pipe_parallel_group()
            last_rank = g.ranks[-1]
            dist.broadcast(loss, src=last_rank, group=g.pg)
        return _wrap(loss)

    def _dp_allreduce(self):
        g = self._dp_group
        if g is None or g.nranks <= 1:
            return
        grads = [p._t.grad for p in self._layers.parameters() if p._t.grad is not None]
        by_dt = {}
        for gr in grads:
            by_dt.setdefault(gr.dtype, []).append(gr)
        for dt, gs in by_dt.items():
            flat = torch.cat([x.reshape(-1) for x in gs])
            dist.all_reduce(flat, group=g.pg)
            flat.div_(g.nranks)
            off = 0
            for x in gs:
                x.copy_(flat[off:off + x.numel()].view_as(x))
                off += x.numel()

    def train_batch(self, data, optimizer, lr_scheduler=None, scaler=None):
        self._layers.train()
        flush = getattr(optimizer, "_flush_grads", None)   # group-sharded stage 1/2 optimizer
        if flush is not None:
            # gradients accumulate over the micro-batches; reduce-scatter once at the end
            with optimizer.no_sync():
                loss = self.forward_backward_pipeline(data, scaler)
            flush()
        else:
            loss = self.forward_backward_pipeline(data, scaler)
        self._dp_allreduce()
        if scaler is not None:
            scaler.step(optimizer)
            scaler.update()
        else:
            optimizer.step()
        optimizer.clear_grad(set_to_zero=False)
        if lr_scheduler is not None:
            lr_scheduler.step()
        return loss

    def eval_batch(self, data, compute_loss=False):
        self._layers.eval()
        with torch.no_grad():
            if self._p2p is None:
                self._p2p = _P2P(self._hcg, self._device())
            p2p = self._p2p
            inputs, labels = data if isinstance(data, (tuple, list)) and len(data) == 2 else (data, None)
            self.total_loss = None
            outs = []
            for i in range(self.accumulate_steps):
                x = self._micro(inputs, i) if self.is_first else None
                if not self.is_first:
                    ts = p2p.recv_forward()
                    x = _wrap(ts[0]) if len(ts) == 1 else tuple(_wrap(t) for t in ts)
                out = self._layers(x)
                if self.is_last:
                    if compute_loss:
                        l = self._layers._loss_fn(out, self._micro(labels, i))
                        l = l._t / self.accumulate_steps
                        self.total_loss = l if self.total_loss is None else self.total_loss + l
                    else:
                        outs.append(out)
                else:
                    p2p.send_forward(_as_list(out))
            if compute_loss:
                return self._broadcast_loss()
            return outs

    def forward(self, *inputs, **kwargs):
        return self._layers(*inputs, **kwargs)
