"""Tensor (model) parallel layers and ops (reference:
python/paddle/distributed/fleet/meta_parallel/parallel_layers/{mp_layers,random}.py,
python/paddle/distributed/collective.py:_c_identity/_c_concat/_c_split/_mp_allreduce/split,
python/paddle/distributed/fleet/layers/mpu/mp_ops.py:_c_softmax_with_cross_entropy).

The TP group is a set of consecutive ranks (GPUs of one node, xGMI-connected). The linear
layers split their rows into pieces (``PHA_TP_OVERLAP_CHUNKS``, default 2) so the all-reduce of
one piece runs on the RCCL stream while the next piece's GEMM (or, in the column layer's
backward, the weight-gradient GEMM) runs on the compute stream.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

from ..framework.core import Tensor, Parameter, _wrap
from ..framework import core as _core
from ..nn.layer.layers import Layer
from ..nn import functional as F
from ..nn import initializer as I
from . import collective as C

__all__ = ["VocabParallelEmbedding", "ColumnParallelLinear", "RowParallelLinear", "ParallelCrossEntropy",
           "RNGStatesTracker", "get_rng_state_tracker", "model_parallel_random_seed", "split",
           "parallel_cross_entropy"]


def _mp_group():
    from . import fleet
    hcg = fleet.fleet._hcg if fleet.fleet._hcg is not None else None
    if hcg is None:
        return None
    return hcg.get_model_parallel_group()


def _pg(group):
    return C._resolve_group(group) if group is not None else None


def _ws(group):
    if group is None:
        return 1
    return group.nranks if isinstance(group, C.Group) else dist.get_world_size(group)


def _rk(group):
    if group is None:
        return 0
    return group.rank if isinstance(group, C.Group) else dist.get_rank(group)


def _static_var(x):
    """x is a static-graph Variable: the TP layer records ONE op (static TP, reference
    fleet/meta_optimizers/tensor_parallel_optimizer.py over paddle.distributed.split)"""
    from ..static import program as P
    return isinstance(x, P.Variable)


def _record(fn, name, args, kwargs):
    from ..static import program as P
    return P.record_op(fn, name, args, kwargs)


def _meta(x, last):
    return _wrap(torch.empty(*x._t.shape[:-1], last, dtype=x._t.dtype, device="meta"))


def column_parallel_linear(x, weight, bias=None, gather_output=True):
    """the op a static ColumnParallelLinear records: x @ W_shard (+ b_shard), optionally gathered"""
    group = _mp_group()
    if x._t.is_meta:
        return _meta(x, weight.shape[1] * (_ws(group) if gather_output else 1))
    xt = x._t
    if _ws(group) > 1 and xt.dim() >= 2:
        y = _wrap(_ColumnParallelMatmul.apply(xt, weight._t, None if bias is None else bias._t, _pg(group),
                                              _tp_chunks(xt.numel() // xt.shape[-1])))
    else:
        y = F.linear(_c_identity(x, group), weight, bias)
    return _c_concat(y, group) if gather_output and _ws(group) > 1 else y


def row_parallel_linear(x, weight, bias=None, input_is_parallel=False):
    """the op a static RowParallelLinear records: all_reduce(x_shard @ W_shard) (+ b)"""
    group = _mp_group()
    if x._t.is_meta:
        return _meta(x, weight.shape[1])
    if not input_is_parallel and _ws(group) > 1:
        x = _c_split(x, group)
    xt = x._t
    if _ws(group) > 1 and xt.dim() >= 2:
        y = _wrap(_RowParallelMatmul.apply(xt, weight._t, _pg(group), _tp_chunks(xt.numel() // xt.shape[-1])))
    else:
        y = _mp_allreduce(F.linear(x, weight, None), group)
    return y + bias if bias is not None else y


def vocab_parallel_embedding(x, weight, vocab_start=0):
    """the op a static VocabParallelEmbedding records: masked local lookup + all_reduce"""
    group = _mp_group()
    if x._t.is_meta:
        return _wrap(torch.empty(*x._t.shape, weight.shape[1], dtype=weight._t.dtype, device="meta"))
    if _ws(group) == 1:
        return F.embedding(x, weight)
    ids = x._t
    per = weight.shape[0]
    mask = (ids < vocab_start) | (ids >= vocab_start + per)
    local = torch.where(mask, torch.zeros_like(ids), ids - vocab_start)
    out = F.embedding(_wrap(local), weight)._t
    out = out.masked_fill(mask.unsqueeze(-1), 0.0)
    return _mp_allreduce(_wrap(out), group)


class _Identity(torch.autograd.Function):
    """c_identity: forward identity, backward all-reduce over the TP group."""

    @staticmethod
    def forward(ctx, x, pg):
        ctx.pg = pg
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        dist.all_reduce(g, group=ctx.pg)
        return g, None


class _AllReduce(torch.autograd.Function):
    """mp_allreduce: forward all-reduce, backward identity."""

    @staticmethod
    def forward(ctx, x, pg):
        x = x.contiguous().clone()
        dist.all_reduce(x, group=pg)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _Split(torch.autograd.Function):
    """c_split along the last dim: forward take my shard, backward all-gather."""

    @staticmethod
    def forward(ctx, x, pg, ws, rk):
        ctx.pg, ctx.ws = pg, ws
        n = x.shape[-1] // ws
        return x[..., rk * n:(rk + 1) * n].contiguous()

    @staticmethod
    def backward(ctx, g):
        return _gather_last(g, ctx.pg, ctx.ws), None, None, None


def _gather_last(x, pg, ws):
    x = x.contiguous()
    outs = [torch.empty_like(x) for _ in range(ws)]
    dist.all_gather(outs, x, group=pg)
    return torch.cat(outs, -1)


class _Concat(torch.autograd.Function):
    """c_concat along the last dim: forward all-gather, backward take my shard."""

    @staticmethod
    def forward(ctx, x, pg, ws, rk):
        ctx.ws, ctx.rk = ws, rk
        return _gather_last(x, pg, ws)

    @staticmethod
    def backward(ctx, g):
        n = g.shape[-1] // ctx.ws
        return g[..., ctx.rk * n:(ctx.rk + 1) * n].contiguous(), None, None, None


def _tp_chunks(rows):
    """token-dim pieces for GEMM / all-reduce overlap (``PHA_TP_OVERLAP_CHUNKS``, default 2; small
    inputs stay whole: a collective's latency would not hide behind a tiny GEMM)"""
    import os
    k = int(os.environ.get("PHA_TP_OVERLAP_CHUNKS", "2"))
    return k if k > 1 and rows >= 256 * k else 1


def _row_splits(rows, k):
    step = -(-rows // k)
    return [(i, min(rows, i + step)) for i in range(0, rows, step)]


class _RowParallelMatmul(torch.autograd.Function):
    """y = all_reduce(x @ W) with the rows in pieces: the all-reduce of piece i runs on the RCCL
    stream while the GEMM of piece i+1 runs on the compute stream (the output buffer is written in
    place, no concat). Backward is local (the all-reduce's gradient is the identity)."""

    @staticmethod
    def forward(ctx, x, w, pg, chunks):
        ctx.save_for_backward(x, w)
        x2 = x.reshape(-1, x.shape[-1])
        y = torch.empty(x2.shape[0], w.shape[1], dtype=x.dtype, device=x.device)
        works = []
        for a, b in _row_splits(x2.shape[0], chunks):
            torch.mm(x2[a:b], w, out=y[a:b])
            works.append(dist.all_reduce(y[a:b], group=pg, async_op=True))
        for wk in works:
            wk.wait()
        return y.reshape(*x.shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = (g2 @ w.t()).reshape(x.shape) if ctx.needs_input_grad[0] else None
        dw = x2.t() @ g2 if ctx.needs_input_grad[1] else None
        return dx, dw, None, None


class _ColumnParallelMatmul(torch.autograd.Function):
    """y = x @ W (+ b) on a column shard; backward: dX = all_reduce(dY W^T) in row pieces whose
    all-reduces overlap the remaining dX pieces and the dW / db GEMMs (the c_identity of the
    input folded into this op)."""

    @staticmethod
    def forward(ctx, x, w, b, pg, chunks):
        ctx.save_for_backward(x, w)
        ctx.pg, ctx.chunks, ctx.has_b = pg, chunks, b is not None
        x2 = x.reshape(-1, x.shape[-1])
        y = torch.addmm(b, x2, w) if b is not None else x2 @ w
        return y.reshape(*x.shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1]).contiguous()
        x2 = x.reshape(-1, x.shape[-1])
        dx, works = None, []
        if ctx.needs_input_grad[0]:
            dx = torch.empty(g2.shape[0], w.shape[0], dtype=g.dtype, device=g.device)
            for a, b in _row_splits(g2.shape[0], ctx.chunks):
                torch.mm(g2[a:b], w.t(), out=dx[a:b])
                works.append(dist.all_reduce(dx[a:b], group=ctx.pg, async_op=True))
        dw = x2.t() @ g2 if ctx.needs_input_grad[1] else None      # overlaps the dX all-reduces
        db = g2.sum(0) if ctx.has_b and ctx.needs_input_grad[2] else None
        for wk in works:
            wk.wait()
        return (dx.reshape(x.shape) if dx is not None else None), dw, db, None, None


def _c_identity(x, group=None):
    group = group if group is not None else _mp_group()
    if _ws(group) == 1:
        return x
    return _wrap(_Identity.apply(x._t, _pg(group)))


def _mp_allreduce(x, group=None):
    group = group if group is not None else _mp_group()
    if _ws(group) == 1:
        return x
    return _wrap(_AllReduce.apply(x._t, _pg(group)))


def _c_split(x, group=None):
    group = group if group is not None else _mp_group()
    if _ws(group) == 1:
        return x
    return _wrap(_Split.apply(x._t, _pg(group), _ws(group), _rk(group)))


def _c_concat(x, group=None):
    group = group if group is not None else _mp_group()
    if _ws(group) == 1:
        return x
    return _wrap(_Concat.apply(x._t, _pg(group), _ws(group), _rk(group)))


class VocabParallelEmbedding(Layer):
    def __init__(self, num_embeddings, embedding_dim, weight_attr=None, mp_group=None, name=None):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _mp_group()
        self.world_size = _ws(self.model_parallel_group)
        self.rank = _rk(self.model_parallel_group)
        self.origin_num_embeddings = num_embeddings
        assert num_embeddings % self.world_size == 0
        self.per_part = num_embeddings // self.world_size
        self.vocab_start_index = self.rank * self.per_part
        with get_rng_state_tracker().rng_state("model_parallel_rng") if self.world_size > 1 else contextlib.nullcontext():
            self.weight = self.create_parameter([self.per_part, embedding_dim], attr=weight_attr,
                                                default_initializer=I.XavierNormal())
        self.weight.is_distributed = self.world_size > 1

    def forward(self, x):
        if _static_var(x):
            return _record(vocab_parallel_embedding, "vocab_parallel_embedding", (x, self.weight),
                           {"vocab_start": int(self.vocab_start_index)})
        if self.world_size == 1:
            return F.embedding(x, self.weight)
        ids = x._t
        lo = self.vocab_start_index
        mask = (ids < lo) | (ids >= lo + self.per_part)
        local = torch.where(mask, torch.zeros_like(ids), ids - lo)
        out = F.embedding(_wrap(local), self.weight)._t
        out = out.masked_fill(mask.unsqueeze(-1), 0)
        return _mp_allreduce(_wrap(out), self.model_parallel_group)


class ColumnParallelLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=None, gather_output=True,
                 fuse_matmul_bias=False, mp_group=None, name=None):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _mp_group()
        self.world_size = _ws(self.model_parallel_group)
        assert out_features % self.world_size == 0
        self.output_size_per_partition = out_features // self.world_size
        self.gather_output = gather_output
        self.in_features, self.out_features = in_features, out_features
        with get_rng_state_tracker().rng_state("model_parallel_rng") if self.world_size > 1 else contextlib.nullcontext():
            self.weight = self.create_parameter([in_features, self.output_size_per_partition], attr=weight_attr)
        self.weight.is_distributed = self.world_size > 1
        if has_bias is None or has_bias:
            self.bias = self.create_parameter([self.output_size_per_partition], is_bias=True)
            self.bias.is_distributed = self.world_size > 1
        else:
            self.bias = None

    def forward(self, x):
        if _static_var(x):
            return _record(column_parallel_linear, "column_parallel_linear", (x, self.weight, self.bias),
                           {"gather_output": bool(self.gather_output)})
        xt = x._t if isinstance(x, Tensor) else x
        if self.world_size > 1 and type(xt).__name__ != "DTensor" and xt.dim() >= 2:
            rows = xt.numel() // xt.shape[-1]
            y = _wrap(_ColumnParallelMatmul.apply(xt, self.weight._t, None if self.bias is None else self.bias._t,
                                                  _pg(self.model_parallel_group), _tp_chunks(rows)))
        else:
            x = _c_identity(x, self.model_parallel_group)
            y = F.linear(x, self.weight, self.bias)
        if self.gather_output and self.world_size > 1:
            y = _c_concat(y, self.model_parallel_group)
        return y


class RowParallelLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=True, input_is_parallel=False,
                 fuse_matmul_bias=False, mp_group=None, name=None):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _mp_group()
        self.world_size = _ws(self.model_parallel_group)
        assert in_features % self.world_size == 0
        self.input_size_per_partition = in_features // self.world_size
        self.input_is_parallel = input_is_parallel
        with get_rng_state_tracker().rng_state("model_parallel_rng") if self.world_size > 1 else contextlib.nullcontext():
            self.weight = self.create_parameter([self.input_size_per_partition, out_features], attr=weight_attr)
        self.weight.is_distributed = self.world_size > 1
        self.bias = self.create_parameter([out_features], is_bias=True) if has_bias else None

    def forward(self, x):
        if _static_var(x):
            return _record(row_parallel_linear, "row_parallel_linear", (x, self.weight, self.bias),
                           {"input_is_parallel": bool(self.input_is_parallel)})
        if not self.input_is_parallel and self.world_size > 1:
            x = _c_split(x, self.model_parallel_group)
        xt = x._t if isinstance(x, Tensor) else x
        if self.world_size > 1 and type(xt).__name__ != "DTensor" and xt.dim() >= 2:
            rows = xt.numel() // xt.shape[-1]
            y = _wrap(_RowParallelMatmul.apply(xt, self.weight._t, _pg(self.model_parallel_group), _tp_chunks(rows)))
        else:
            y = F.linear(x, self.weight, None)
            y = _mp_allreduce(y, self.model_parallel_group)
        if self.bias is not None:
            y = y + self.bias
        return y


class _ParallelCE(torch.autograd.Function):
    """Softmax CE over vocab-sharded logits (reference: c_softmax_with_cross_entropy_op.cu)."""

    @staticmethod
    def forward(ctx, logits, labels, pg, rank, ignore_index):
        V = logits.shape[-1]
        lo = rank * V
        x = logits.float()
        m = x.max(-1, keepdim=True).values
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=pg)
        e = torch.exp(x - m)
        s = e.sum(-1, keepdim=True)
        dist.all_reduce(s, group=pg)
        lab = labels.long()
        inside = (lab >= lo) & (lab < lo + V)
        idx = torch.where(inside, lab - lo, torch.zeros_like(lab))
        tgt = torch.gather(x, -1, idx.unsqueeze(-1)).squeeze(-1)
        tgt = torch.where(inside, tgt, torch.zeros_like(tgt))
        dist.all_reduce(tgt, group=pg)
        loss = torch.log(s.squeeze(-1)) + m.squeeze(-1) - tgt
        valid = lab != ignore_index
        loss = torch.where(valid, loss, torch.zeros_like(loss))
        softmax = e / s
        ctx.save_for_backward(softmax, idx, inside & valid, valid)
        ctx.dtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, g):
        softmax, idx, hit, valid = ctx.saved_tensors
        grad = softmax.clone()
        onehot = torch.zeros_like(grad).scatter_(-1, idx.unsqueeze(-1), hit.unsqueeze(-1).to(grad.dtype))
        grad = (grad - onehot) * (g * valid.to(g.dtype)).unsqueeze(-1)
        return grad.to(ctx.dtype), None, None, None, None


def parallel_cross_entropy(logits, labels, group=None, ignore_index=-100):
    group = group if group is not None else _mp_group()
    if _ws(group) == 1:
        from .. import ops
        return ops.softmax_cross_entropy(logits, labels, ignore_index)
    return _ParallelCE.apply(logits, labels, _pg(group), _rk(group), ignore_index)


class ParallelCrossEntropy(Layer):
    def __init__(self, mp_group=None, name=None, ignore_index=-100):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _mp_group()
        self.ignore_index = ignore_index

    def forward(self, input, label):
        lab = label._t
        if lab.dim() == input._t.dim():
            lab = lab.squeeze(-1)
        loss = parallel_cross_entropy(input._t, lab, self.model_parallel_group, self.ignore_index)
        return _wrap(loss.unsqueeze(-1))


# ----------------------------------------------------------------------------- RNG tracker
class RNGStatesTracker:
    """Named RNG states so TP shards draw different dropout masks / inits while DP replicas agree."""

    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def add(self, name, seed):
        if seed in self.seeds_:
            raise ValueError(f"seed {seed} already exists")
        self.seeds_.add(seed)
        if name in self.states_:
            raise ValueError(f"state {name} already exists")
        cur = _get_state()
        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed(seed)
        self.states_[name] = _get_state()
        _set_state(cur)

    def get_states_tracker(self):
        return dict(self.states_)

    def set_states_tracker(self, states):
        self.states_ = dict(states)

    @contextlib.contextmanager
    def rng_state(self, name="model_parallel_rng"):
        if name not in self.states_:
            yield
            return
        orig = _get_state()
        _set_state(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = _get_state()
            _set_state(orig)


def _get_state():
    s = {"cpu": torch.get_rng_state()}
    if torch.cuda.is_available():
        s["cuda"] = torch.cuda.get_rng_state()
    return s


def _set_state(s):
    torch.set_rng_state(s["cpu"])
    if "cuda" in s and torch.cuda.is_available():
        torch.cuda.set_rng_state(s["cuda"])


_tracker = RNGStatesTracker()


def get_rng_state_tracker():
    return _tracker


def model_parallel_random_seed(seed=None):
    from . import fleet
    hcg = fleet.fleet._hcg
    rank = hcg.get_model_parallel_rank() if hcg is not None else 0
    import random
    seed = seed if seed is not None else random.randint(0, 2 ** 20)
    local_seed = seed + 1024 + rank * 100
    global_seed = seed
    _tracker.reset()
    _tracker.add("global_seed", global_seed)
    _tracker.add("local_seed", local_seed)
    _tracker.add("model_parallel_rng", local_seed + 1)
    torch.manual_seed(global_seed)


def split(x, size, operation, axis=0, num_partitions=1, gather_out=True, weight_attr=None, bias_attr=None, name=None):
    """paddle.distributed.split: build a TP linear/embedding on the fly and apply it."""
    if operation == "embedding":
        layer = VocabParallelEmbedding(size[0], size[1], weight_attr=weight_attr)
        return layer(x)
    if operation == "linear":
        if axis == 0:
            layer = RowParallelLinear(size[0], size[1], weight_attr=weight_attr, has_bias=bias_attr is not False,
                                      input_is_parallel=False)
        else:
            layer = ColumnParallelLinear(size[0], size[1], weight_attr=weight_attr, has_bias=bias_attr is not False,
                                         gather_output=gather_out)
        return layer(x)
    raise ValueError(operation)
