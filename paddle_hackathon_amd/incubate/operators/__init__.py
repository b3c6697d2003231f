"""Graph-learning and fused-softmax operators (reference: python/paddle/incubate/operators/
graph_*.py, softmax_mask_fuse*.py; python/paddle/incubate/tensor/math.py segment_*).

Message passing (``graph_send_recv``) and segment reductions run as one gather plus one
``scatter_reduce`` on the device. Neighbour sampling/reindexing is irregular, pointer-chasing
work and runs on the host over the CSC arrays (as the reference's CPU kernels do)."""
from __future__ import annotations

import numpy as np
import torch

from ...framework.core import Tensor, _wrap
from ...framework.dispatch import register_ops
from ... import ops as _ops

__all__ = ["graph_send_recv", "graph_khop_sampler", "graph_reindex", "graph_sample_neighbors", "segment_sum",
           "segment_mean", "segment_max", "segment_min", "softmax_mask_fuse", "softmax_mask_fuse_upper_triangle",
           "identity_loss"]


def _u(x):
    return x._t if isinstance(x, Tensor) else torch.as_tensor(x)


_REDUCE = {"sum": "sum", "mean": "mean", "max": "amax", "min": "amin"}


def _scatter(src, index, n, pool):
    pool = pool.lower()
    if pool not in _REDUCE:
        raise ValueError(f"pool_type should be sum/mean/max/min, got {pool}")
    shape = (n,) + tuple(src.shape[1:])
    out = torch.zeros(shape, dtype=src.dtype, device=src.device)
    idx = index.long().reshape(-1, *([1] * (src.dim() - 1))).expand_as(src)
    out = out.scatter_reduce(0, idx, src, reduce=_REDUCE[pool], include_self=False)
    return out


def graph_send_recv(x, src_index, dst_index, pool_type="sum", out_size=None, name=None):
    t = _u(x)
    n = t.shape[0] if out_size is None or (isinstance(out_size, int) and out_size <= 0) else \
        int(out_size if isinstance(out_size, int) else _u(out_size).reshape(-1)[0].item())
    return _wrap(_scatter(t[_u(src_index).long()], _u(dst_index), n, pool_type))


def _segment(data, segment_ids, pool):
    t = _u(data)
    ids = _u(segment_ids)
    n = int(ids.max().item()) + 1 if ids.numel() else 0
    return _wrap(_scatter(t, ids, n, pool))


def segment_sum(data, segment_ids, name=None):
    return _segment(data, segment_ids, "sum")


def segment_mean(data, segment_ids, name=None):
    return _segment(data, segment_ids, "mean")


def segment_max(data, segment_ids, name=None):
    return _segment(data, segment_ids, "max")


def segment_min(data, segment_ids, name=None):
    return _segment(data, segment_ids, "min")


def _np(x):
    return x.numpy() if isinstance(x, Tensor) else np.asarray(x)


def graph_sample_neighbors(row, colptr, input_nodes, eids=None, perm_buffer=None, sample_size=-1, return_eids=False,
                           flag_perm_buffer=False, name=None):
    """Uniformly sample up to ``sample_size`` in-neighbours of each input node (CSC graph)."""
    r, cp, nodes = _np(row), _np(colptr), _np(input_nodes)
    e = _np(eids) if eids is not None else None
    if return_eids and e is None:
        raise ValueError("eids should not be None if return_eids is True")
    rng = np.random.default_rng(int(torch.randint(0, 2 ** 31, (1,)).item()))
    outs, counts, out_e = [], [], []
    for n in nodes:
        beg, end = int(cp[n]), int(cp[n + 1])
        deg = end - beg
        if sample_size < 0 or deg <= sample_size:
            sel = np.arange(beg, end)
        else:
            sel = beg + rng.choice(deg, sample_size, replace=False)
        outs.append(r[sel])
        counts.append(len(sel))
        if return_eids:
            out_e.append(e[sel])
    dev = _u(row).device if isinstance(row, Tensor) else None
    mk = lambda a, dt: _wrap(torch.as_tensor(np.concatenate(a) if a else np.zeros(0, dt), device=dev))  # noqa: E731
    res = (mk(outs, r.dtype), _wrap(torch.as_tensor(np.asarray(counts, dtype=np.int32), device=dev)))
    if return_eids:
        return res + (mk(out_e, e.dtype),)
    return res


def _reindex(x, neighbors, count):
    order = {}
    out_nodes = []
    for v in x.tolist():
        if v not in order:
            order[v] = len(out_nodes)
            out_nodes.append(v)
    src = np.empty(len(neighbors), dtype=np.int64)
    for i, v in enumerate(neighbors.tolist()):
        j = order.get(v)
        if j is None:
            j = order[v] = len(out_nodes)
            out_nodes.append(v)
        src[i] = j
    dst = np.repeat(np.arange(len(x), dtype=np.int64), count)
    return src, dst, np.asarray(out_nodes, dtype=x.dtype)


def graph_reindex(x, neighbors, count, value_buffer=None, index_buffer=None, flag_buffer_hashtable=False, name=None):
    xs, nb, ct = _np(x), _np(neighbors), _np(count)
    src, dst, nodes = _reindex(xs, nb, ct)
    dev = _u(x).device if isinstance(x, Tensor) else None
    dt = torch.as_tensor(xs[:0]).dtype
    return (_wrap(torch.as_tensor(src, device=dev).to(dt)), _wrap(torch.as_tensor(dst, device=dev).to(dt)),
            _wrap(torch.as_tensor(nodes, device=dev)))


def graph_khop_sampler(row, colptr, input_nodes, sample_sizes, sorted_eids=None, return_eids=False, name=None):
    """Multi-hop sampling; returns (edge_src, edge_dst, sample_index, reindex_nodes[, edge_eids])."""
    nodes = _np(input_nodes)
    frontier = nodes
    all_src, all_dst, all_e = [], [], []
    for k in sample_sizes:
        res = graph_sample_neighbors(row, colptr, frontier, sorted_eids, None, k, return_eids)
        nb, ct = _np(res[0]), _np(res[1])
        all_src.append(nb)
        all_dst.append(np.repeat(frontier, ct))
        if return_eids:
            all_e.append(_np(res[2]))
        frontier = np.unique(nb)
    src = np.concatenate(all_src) if all_src else np.zeros(0, nodes.dtype)
    dst = np.concatenate(all_dst) if all_dst else np.zeros(0, nodes.dtype)
    order, sample = {}, []
    for v in list(nodes.tolist()) + list(dst.tolist()) + list(src.tolist()):
        if v not in order:
            order[v] = len(sample)
            sample.append(v)
    rs = np.asarray([order[v] for v in src.tolist()], dtype=np.int64)
    rd = np.asarray([order[v] for v in dst.tolist()], dtype=np.int64)
    reidx = np.asarray([order[v] for v in nodes.tolist()], dtype=np.int64)
    dev = _u(row).device if isinstance(row, Tensor) else None
    dt = torch.as_tensor(nodes[:0]).dtype
    w = lambda a: _wrap(torch.as_tensor(a, device=dev).to(dt))  # noqa: E731
    out = (w(rs.reshape(-1, 1)), w(rd.reshape(-1, 1)), w(np.asarray(sample, dtype=np.int64)), w(reidx))
    if return_eids:
        return out + (_wrap(torch.as_tensor(np.concatenate(all_e) if all_e else np.zeros(0, np.int64), device=dev)),)
    return out


def softmax_mask_fuse(x, mask, name=None):
    """softmax(x + mask) over the last axis; the add is folded into the HIP softmax input."""
    t, m = _u(x), _u(mask)
    return _wrap(_ops.fused.softmax((t + m).contiguous(), -1))


def softmax_mask_fuse_upper_triangle(x):
    """Causal softmax: entries above the diagonal of the last two dims are masked out."""
    t = _u(x)
    S, T = t.shape[-2], t.shape[-1]
    causal = torch.ones(S, T, dtype=torch.bool, device=t.device).triu(1)
    return _wrap(_ops.fused.softmax(t.masked_fill(causal, float("-inf")).contiguous(), -1))


def identity_loss(x, reduction="none"):
    if isinstance(reduction, str):
        reduction = {"sum": 0, "mean": 1, "none": 2}.get(reduction.lower(), reduction)
    t = _u(x)
    if reduction == 0:
        return _wrap(t.sum())
    if reduction == 1:
        return _wrap(t.mean())
    if reduction == 2:
        return _wrap(t)
    raise ValueError(f"unsupported reduction {reduction}")


register_ops(globals(), __all__)


from .resnet_unit import ResNetUnit, resnet_unit  # noqa: E402,F401

__all__ += ["ResNetUnit", "resnet_unit"]
