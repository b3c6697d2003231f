"""Hybrid-parallel gradient / parameter synchronisation helpers (reference:
python/paddle/distributed/fleet/utils/hybrid_parallel_util.py:111-199 — broadcast_input_data,
broadcast_mp_parameters, broadcast_dp_parameters, fused_allreduce_gradients,
sharding_reduce_gradients, broadcast_sharding_parameters). fleetx / PaddleNLP training loops
call these directly around a manual ``loss.backward()``.

MI355X design. ``fused_allreduce_gradients`` coalesces the gradients into buckets of one dtype
(128 MB, as the reference; over xGMI rings a few large all-reduces reach the per-link bandwidth,
many small ones stay latency-bound), pre-scales each flat bucket by 1 / nranks in place and
all-reduces it with one RCCL call per bucket on the current stream, then scatters it back through
views — no per-tensor collectives, no host round trips. The scale happens before the sum so bf16
buckets do not overflow at large data-parallel degrees, as the reference does."""
from __future__ import annotations

import torch

from ... import collective as C
from ...data_parallel import sync_params_buffers

__all__ = ["broadcast_input_data", "broadcast_mp_parameters", "broadcast_dp_parameters", "fused_allreduce_gradients",
           "sharding_reduce_gradients", "broadcast_sharding_parameters"]

_BUCKET_BYTES = 128 * 1024 * 1024


def _grads(parameter_list):
    out, seen = [], set()
    for p in parameter_list:
        t = getattr(p, "_t", p)
        if getattr(p, "trainable", True) and not getattr(p, "stop_gradient", False) and t.grad is not None:
            g = t.grad
            if g.is_sparse:
                raise NotImplementedError("fused_allreduce_gradients: sparse gradients are not supported")
            if id(g) in seen:
                raise AssertionError("a gradient is shared by two parameters")
            seen.add(id(g))
            out.append(g)
    return out


def _buckets(grads, limit=_BUCKET_BYTES):
    """consecutive gradients of one dtype and device, up to ``limit`` bytes per bucket"""
    out, cur, size = [], [], 0
    for g in grads:
        nb = g.numel() * g.element_size()
        if cur and (size + nb > limit or g.dtype != cur[0].dtype or g.device != cur[0].device):
            out.append(cur)
            cur, size = [], 0
        cur.append(g)
        size += nb
    if cur:
        out.append(cur)
    return out


def _allreduce_mean(grads, group):
    pg = C._resolve_group(group)
    nranks = C._nranks(group) if group is not None else C.get_world_size()
    if nranks <= 1:
        return
    import torch.distributed as dist
    with torch.no_grad():
        for bucket in _buckets(grads):
            flat = torch.cat([g.reshape(-1) for g in bucket]) if len(bucket) > 1 else bucket[0].reshape(-1)
            flat.mul_(1.0 / nranks)
            dist.all_reduce(flat, group=pg)
            if len(bucket) > 1 or flat.data_ptr() != bucket[0].data_ptr():
                off = 0
                for g in bucket:
                    n = g.numel()
                    g.copy_(flat[off:off + n].view_as(g))
                    off += n


def fused_allreduce_gradients(parameter_list, hcg):
    """mean of every parameter gradient over the data-parallel group (the whole world without hcg)"""
    group = None if hcg is None else hcg.get_data_parallel_group()
    _allreduce_mean(_grads(parameter_list), group)


def sharding_reduce_gradients(parameter_list, hcg):
    """mean of the gradients over the sharding group (the reference all-reduces too: every rank
    keeps the full gradient before its optimizer shard steps)"""
    _allreduce_mean(_grads(parameter_list), hcg.get_sharding_parallel_group())


def broadcast_mp_parameters(model, hcg):
    """replicated (non ``is_distributed``) parameters from the model-parallel group's first rank"""
    sync_params_buffers(model, hcg.get_model_parallel_group(), 0, is_model_parallel=True)   # group rank 0


def broadcast_dp_parameters(model, hcg):
    sync_params_buffers(model, hcg.get_data_parallel_group(), 0, is_model_parallel=False)


def broadcast_sharding_parameters(model, hcg):
    sync_params_buffers(model, hcg.get_sharding_parallel_group(), 0, is_model_parallel=False)


def _broadcast_data(t, hcg):
    import torch.distributed as dist
    group = hcg.get_model_parallel_group()
    if C._nranks(group) <= 1:
        return
    pg = C._resolve_group(group)
    src = hcg.get_model_parallel_group_src_rank()   # the group's first rank, a global rank
    with torch.no_grad():
        dist.broadcast(t._t if hasattr(t, "_t") else t, src=src, group=pg)


def broadcast_input_data(hcg, *inputs, **kwargs):
    """every model-parallel rank sees the first rank's batch (inputs are overwritten in place)"""
    from ....framework.core import Tensor
    for v in inputs:
        if isinstance(v, (Tensor, torch.Tensor)):
            _broadcast_data(v, hcg)
    for k, v in kwargs.items():
        if isinstance(v, (Tensor, torch.Tensor)):
            _broadcast_data(v, hcg)
    return inputs, kwargs
