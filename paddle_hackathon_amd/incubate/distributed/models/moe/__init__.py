"""Mixture-of-Experts with expert parallelism (reference: python/paddle/incubate/distributed/
models/moe/{moe_layer,gate/*,grad_clip}.py).

Forward: gate → top-k expert ids (+ capacity limit) → sort token-slots by global expert →
uneven all-to-all (RCCL) so every rank receives the tokens of its local experts → regroup
received rows by local expert → run experts on contiguous slices → inverse regroup →
all-to-all back → unsort → combine the top-k outputs weighted by the gate values.
On MI355X pick the EP degree so each all-to-all moves ≥ a few MB per peer: xGMI is
point-to-point, and per-peer messages below that are latency bound."""
from __future__ import annotations

import math

import torch

from .....framework.core import Tensor, _wrap
from .....nn.layer.layers import Layer
from ..... import nn
from .....nn.clip import ClipGradByGlobalNorm
from .utils import (count_by_gate, limit_by_capacity, _random_routing, _A2A, _nranks,  # noqa: F401
                    global_scatter, global_gather)

__all__ = ["MoELayer", "BaseGate", "NaiveGate", "GShardGate", "SwitchGate", "ClipGradForMOEByGlobalNorm",
           "ClipGradByGlobalNorm"]


class BaseGate(Layer):
    def __init__(self, num_expert, world_size):
        super().__init__()
        self.world_size = world_size
        self.num_expert = num_expert
        self.tot_expert = world_size * num_expert
        self.loss = None

    def forward(self, x):
        raise NotImplementedError

    def set_loss(self, loss):
        self.loss = loss

    def get_loss(self, clear=True):
        loss = self.loss
        if clear:
            self.loss = None
        return loss


class NaiveGate(BaseGate):
    def __init__(self, d_model, num_expert, world_size, topk=2):
        super().__init__(num_expert, world_size)
        self.gate = nn.Linear(d_model, self.tot_expert)
        self.top_k = topk

    def forward(self, inp, return_all_scores=False):
        score = self.gate(inp)._t
        val, idx = torch.topk(score, self.top_k, dim=-1, largest=True, sorted=False)
        if return_all_scores:
            return _wrap(val), _wrap(idx), _wrap(score)
        return _wrap(val), _wrap(idx)


class GShardGate(NaiveGate):
    def __init__(self, d_model, num_expert, world_size, topk=2, capacity=(1.2, 2.4), random_routing=True, group=None):
        if topk != 2:
            raise ValueError("topk should be 2 in gshard")
        super().__init__(d_model, num_expert, world_size)
        self.capacity, self.random_routing, self.group = capacity, random_routing, group

    def forward(self, x):
        val, idx, score = super().forward(x, return_all_scores=True)
        v, i, s = val._t, idx._t, score._t
        n = s.shape[0]
        c_e = torch.bincount(i.reshape(-1), minlength=self.tot_expert).float() / n
        m_e = torch.softmax(s.float(), 1).mean(0)
        self.set_loss(_wrap((c_e * m_e).mean() * (self.num_expert ** 2)))
        cap = math.ceil(self.capacity[0 if self.training else 1] * x.shape[0])
        _, _, i = limit_by_capacity(i, self.num_expert, self.world_size, cap, self.group)
        if self.random_routing:
            i = _random_routing(i, v, torch.rand(n, device=v.device))
        return _wrap(v), _wrap(i)


class SwitchGate(NaiveGate):
    def __init__(self, d_model, num_expert, world_size, topk=1, switch_eps=0.1, capacity=(1.2, 2.4), group=None):
        if topk != 1:
            raise ValueError("topk should be 1 in switch")
        super().__init__(d_model, num_expert, world_size, topk=1)
        self.switch_eps, self.capacity, self.group = switch_eps, capacity, group

    def forward(self, inp):
        score = self.gate(inp)._t
        if self.training:
            score = score + (torch.rand_like(score) * 2 * self.switch_eps + 1.0 - self.switch_eps)
        score = torch.softmax(score, -1)
        v, i = torch.topk(score, 1, dim=-1)
        cap = math.ceil(self.capacity[0 if self.training else 1] * inp.shape[0])
        _, _, i = limit_by_capacity(i, self.num_expert, self.world_size, cap, self.group)
        valid = i[i > -1]
        frac = torch.bincount(valid, minlength=self.tot_expert).float() / max(valid.numel(), 1)
        prob = score.sum(0) / max(valid.numel(), 1)
        self.set_loss(_wrap((frac * prob).sum() * self.tot_expert))
        return _wrap(v), _wrap(i)


class MoELayer(Layer):
    def __init__(self, d_model, experts, gate=None, moe_group=None, mp_group=None, **kwargs):
        super().__init__()
        self.recompute_interval = kwargs.get("recompute_interval", 0)
        gate = {} if gate is None else gate
        self.group = moe_group
        self.world_size = moe_group.nranks if moe_group is not None else 1
        self.num_expert = len(experts)
        self.experts = experts
        self.mp_group = mp_group
        self.d_model = d_model
        if isinstance(gate, dict):
            self.top_k = gate.get("top_k", 2)
            kind = gate.get("type", "gshard")
            if kind in ("naive", None):
                gate = NaiveGate(d_model, self.num_expert, self.world_size, self.top_k)
            elif kind == "gshard":
                gate = GShardGate(d_model, self.num_expert, self.world_size, self.top_k, group=self.group)
            elif kind == "switch":
                gate = SwitchGate(d_model, self.num_expert, self.world_size, self.top_k, group=self.group)
            else:
                raise ValueError(f"unsupported gate type {kind}")
        elif isinstance(gate, NaiveGate):
            self.top_k = gate.top_k
        else:
            raise TypeError("gate must be a dict or a NaiveGate/GShardGate/SwitchGate")
        self.gate = gate

    def _experts_fwd(self, x, counts):
        outs, start = [], 0
        for e, c in enumerate(counts):
            if c > 0:
                outs.append(self.experts[e](_wrap(x[start:start + c]))._t)
            start += c
        return torch.cat(outs, 0) if outs else x[:0]

    def forward(self, inp):
        if len(inp.shape) != 3:
            raise ValueError("MoELayer input must be [batch, seq, d_model]")
        origin = inp.shape
        x = inp._t.reshape(-1, origin[2])
        mp_size = self.mp_group.nranks if self.mp_group is not None else 1
        if mp_size > 1:  # each mp rank routes a slice of the tokens
            chunk = x.shape[0] // mp_size
            x = x[self.mp_group.rank * chunk:(self.mp_group.rank + 1) * chunk]
        value, gate_idx = self.gate(_wrap(x))
        v, gi = value._t, gate_idx._t
        topk = gi.shape[1] if gi.dim() == 2 else 1
        W, E = self.world_size, self.num_expert
        pos, lec, gec = count_by_gate(gi, E, W, self.group)
        rows = x[torch.div(pos, topk, rounding_mode="floor")]  # token rows, sorted by global expert
        send = lec.reshape(W, E).sum(1).tolist()
        gec_cpu = gec.reshape(W, E).cpu()
        recv = gec_cpu.sum(1).tolist()
        y = _A2A.apply(rows, send, recv, self.group) if W > 1 else rows
        # received rows are [src rank][local expert]; regroup to [local expert][src rank]
        if W > 1:
            starts = torch.cumsum(torch.cat([torch.zeros(1, dtype=torch.long), gec_cpu.reshape(-1)]), 0)[:-1]
            perm = torch.cat([torch.arange(int(starts[r * E + e]), int(starts[r * E + e] + gec_cpu[r, e]))
                              for e in range(E) for r in range(W)]) if y.shape[0] else torch.zeros(0, dtype=torch.long)
            perm = perm.to(y.device)
            y = y[perm]
        counts = gec_cpu.sum(0).tolist()
        if self.recompute_interval > 0 and self.training and y.shape[0]:
            from .....parallel.recompute import recompute
            y = recompute(lambda t: _wrap(self._experts_fwd(t._t, counts)), _wrap(y))._t
        else:
            y = self._experts_fwd(y, counts)
        if W > 1:
            inv = torch.empty_like(perm)
            inv[perm] = torch.arange(perm.numel(), device=perm.device)
            y = y[inv]
            y = _A2A.apply(y, recv, send, self.group)
        # unsort back to (token, slot) order; dropped slots contribute zero
        out = y.new_zeros((x.shape[0] * topk, self.d_model))
        out = out.index_copy(0, pos, y)
        out = out.reshape(-1, topk, self.d_model)
        keep = (gi.reshape(-1, topk) >= 0).to(v.dtype)
        w = (v.reshape(-1, 1, topk) * keep.reshape(-1, 1, topk)).to(out.dtype)
        res = torch.bmm(w, out).reshape(-1, self.d_model)
        if mp_size > 1:
            res = _AllGatherRows.apply(res, self.mp_group)
        return _wrap(res.reshape(origin))


class _AllGatherRows(torch.autograd.Function):
    """Concatenate row slices from every rank of ``group`` (grad: take own slice)."""

    @staticmethod
    def forward(ctx, x, group):
        import torch.distributed as dist
        from .....parallel import collective as C
        ctx.group = group
        parts = [torch.empty_like(x) for _ in range(group.nranks)]
        dist.all_gather(parts, x.contiguous(), group=C._resolve_group(group))
        return torch.cat(parts, 0)

    @staticmethod
    def backward(ctx, g):
        n = g.shape[0] // ctx.group.nranks
        return g[ctx.group.rank * n:(ctx.group.rank + 1) * n], None


class ClipGradForMOEByGlobalNorm(ClipGradByGlobalNorm):
    """Global-norm clip where expert parameters' squared norms are summed across the MoE
    group (they are distinct per rank) and the rest are counted once."""

    def __init__(self, clip_norm, is_expert_param_func=None, moe_group=None, group_name="default_moe_group"):
        super().__init__(clip_norm)
        self.is_expert_param_func = is_expert_param_func
        self.moe_group = moe_group

    def _dygraph_clip(self, params_grads):
        import torch.distributed as dist
        normal, expert = [], []
        for p, g in params_grads:
            if g is None or getattr(p, "need_clip", True) is False:
                continue
            (expert if self.is_expert_param_func is not None and self.is_expert_param_func(p) else normal).append(g._t)
        dev = (normal or expert)[0].device if (normal or expert) else torch.device("cpu")
        sq = lambda gs: sum((x.float() ** 2).sum() for x in gs) if gs else torch.zeros((), device=dev)  # noqa: E731
        e = sq(expert)
        if self.moe_group is not None and self.moe_group.nranks > 1:
            from .....parallel import collective as C
            dist.all_reduce(e, group=C._resolve_group(self.moe_group))
        norm = torch.sqrt(sq(normal) + e)
        scale = torch.clamp(self.clip_norm / torch.clamp(norm, min=1e-6), max=1.0)
        out = []
        for p, g in params_grads:
            if g is None or getattr(p, "need_clip", True) is False:
                out.append((p, g))
                continue
            out.append((p, _wrap((g._t.float() * scale).to(g._t.dtype))))
        return out

    def __call__(self, params_grads):
        return self._dygraph_clip(params_grads)
