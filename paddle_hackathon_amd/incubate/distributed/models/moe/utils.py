"""Expert-parallel token exchange (reference: python/paddle/incubate/distributed/models/moe/
utils.py, moe_layer.py MoEScatter/MoEGather, python/paddle/distributed/utils.py
global_scatter/global_gather and the CUDA ops number_count/assign_pos/limit_by_capacity).

Layout: ``tot_expert = num_expert * world_size`` experts, global expert id
``g = rank * num_expert + e``. Tokens are sorted by global expert id, so the rows bound for
one rank are contiguous, and exchanged with ONE uneven all-to-all (RCCL all_to_all_single
over xGMI) per direction. Counts are exchanged first with a tiny all-to-all."""
from __future__ import annotations

import torch
import torch.distributed as dist

from .....parallel import collective as C


def _pg(group):
    return C._resolve_group(group) if group is not None else None


def _nranks(group):
    if group is None:
        return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    return group.nranks


def _my_rank(group):
    if group is None:
        return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    return group.rank


def a2a_uneven(x, in_splits, out_splits, group=None):
    """all_to_all_single with per-rank row counts (lists of ints)."""
    n = _nranks(group)
    if n == 1:
        return x.clone()
    out = x.new_empty((sum(out_splits),) + tuple(x.shape[1:]))
    if dist.get_backend(_pg(group)) == "gloo":
        ins = list(torch.split(x.contiguous(), in_splits))
        outs = list(torch.split(out, out_splits))
        me = _my_rank(group)
        ranks = group.ranks if group is not None else list(range(n))
        ops = []
        for r in range(n):
            if r == me:
                outs[r].copy_(ins[r])
                continue
            if ins[r].numel():
                ops.append(dist.P2POp(dist.isend, ins[r].contiguous(), ranks[r], _pg(group)))
            if outs[r].numel():
                ops.append(dist.P2POp(dist.irecv, outs[r], ranks[r], _pg(group)))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return torch.cat(outs) if outs else out
    dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits, group=_pg(group))
    return out


class _A2A(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, in_splits, out_splits, group):
        ctx.in_splits, ctx.out_splits, ctx.group = in_splits, out_splits, group
        return a2a_uneven(x, in_splits, out_splits, group)

    @staticmethod
    def backward(ctx, g):
        return a2a_uneven(g.contiguous(), ctx.out_splits, ctx.in_splits, ctx.group), None, None, None


def count_by_gate(gate_idx, num_expert, world_size, group=None):
    """Returns (pos, local_expert_count[tot], global_expert_count[world, num_expert]).
    ``pos`` lists flattened (token, slot) indices sorted by expert; dropped slots (-1) excluded."""
    flat = gate_idx.reshape(-1)
    tot = num_expert * world_size
    valid = flat >= 0
    key = torch.where(valid, flat, torch.full_like(flat, tot))
    pos = torch.argsort(key, stable=True)[: int(valid.sum().item())]
    lec = torch.bincount(flat[valid].long(), minlength=tot)
    if world_size > 1:
        gec = a2a_uneven(lec.reshape(world_size, num_expert), [1] * world_size, [1] * world_size, group)
    else:
        gec = lec.reshape(1, num_expert).clone()
    return pos, lec, gec


def limit_by_capacity(topk_idx, num_expert, world_size, capacity, group=None):
    """Drop (set to -1) assignments beyond ``capacity`` tokens per global expert, in token order.
    With world_size > 1 the capacity is shared across the ranks sending to an expert: each
    rank's quota is granted in rank order (reference limit_by_capacity + prune_gate_by_capacity)."""
    flat = topk_idx.reshape(-1).long()
    tot = num_expert * world_size
    lec = torch.bincount(flat[flat >= 0], minlength=tot)
    if world_size > 1:
        allc = [torch.zeros_like(lec) for _ in range(world_size)]
        dist.all_gather(allc, lec, group=_pg(group))
        allc = torch.stack(allc)  # [world, tot]
        before = allc[: _my_rank(group)].sum(0)
        quota = (capacity - before).clamp_min(0)
    else:
        quota = torch.full((tot,), capacity, dtype=lec.dtype, device=lec.device)
    # rank of each assignment among those to the same expert (stable token order)
    out = flat.clone()
    order = torch.argsort(torch.where(flat >= 0, flat, torch.full_like(flat, tot)), stable=True)
    sorted_e = flat[order]
    ok = sorted_e >= 0
    first = torch.zeros(tot + 1, dtype=torch.long, device=flat.device)
    counts = torch.bincount(sorted_e[ok], minlength=tot)
    first[1:] = torch.cumsum(counts, 0)
    idx_in_e = torch.arange(order.numel(), device=flat.device) - first[sorted_e.clamp_min(0)]
    drop = ok & (idx_in_e >= quota[sorted_e.clamp_min(0)])
    out[order[drop]] = -1
    new_lec = torch.bincount(out[out >= 0], minlength=tot)
    return new_lec, None, out.reshape(topk_idx.shape).to(topk_idx.dtype)


def _random_routing(topk_idx, topk_value, prob, topk=2):
    """GShard second-expert random routing: drop slot 1 when 2*value < prob."""
    if topk != 2:
        raise ValueError("random routing needs top-2")
    out = topk_idx.clone()
    drop = 2 * topk_value[:, 1] < prob
    out[:, 1] = torch.where(drop, torch.full_like(out[:, 1], -1), out[:, 1])
    return out


def global_scatter(x, local_count, global_count, group=None, use_calc_stream=True):
    """Send rows of ``x`` (sorted by global expert) to the ranks owning the experts.
    local_count: [world*num_expert]; global_count: [world*num_expert] (rows I receive)."""
    from .....framework.core import Tensor, _wrap
    t = x._t if isinstance(x, Tensor) else x
    lc = (local_count._t if isinstance(local_count, Tensor) else local_count).long()
    gc = (global_count._t if isinstance(global_count, Tensor) else global_count).long()
    w = _nranks(group)
    ins = lc.reshape(w, -1).sum(1).tolist()
    outs = gc.reshape(w, -1).sum(1).tolist()
    return _wrap(_A2A.apply(t, ins, outs, group))


def global_gather(x, local_count, global_count, group=None, use_calc_stream=True):
    """Inverse of :func:`global_scatter`."""
    from .....framework.core import Tensor, _wrap
    t = x._t if isinstance(x, Tensor) else x
    lc = (local_count._t if isinstance(local_count, Tensor) else local_count).long()
    gc = (global_count._t if isinstance(global_count, Tensor) else global_count).long()
    w = _nranks(group)
    return _wrap(_A2A.apply(t, gc.reshape(w, -1).sum(1).tolist(), lc.reshape(w, -1).sum(1).tolist(), group))
