"""Sparse functional ops (reference: python/paddle/incubate/sparse/nn/functional/*.py).

Sparse 3-D convolution uses a gather-GEMM-scatter formulation: for each kernel offset the
active input sites are matched to output sites through a hash of voxel coordinates, their
features are gathered into one dense [M, Cin] matrix and multiplied by the [Cin, Cout]
kernel slice (a dense GEMM on the MFMA units), and the products are scatter-added into
the outputs. Submanifold conv keeps the output sites equal to the input sites."""
from __future__ import annotations

import itertools

import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _wrap

__all__ = ["conv3d", "subm_conv3d", "max_pool3d", "relu", "relu6", "leaky_relu", "softmax", "attention"]


def _vals(x, fn):
    t = x._t
    if t.is_sparse:
        c = t.coalesce()
        return _wrap(torch.sparse_coo_tensor(c.indices(), fn(c.values()), c.shape, is_coalesced=True))
    if t.layout == torch.sparse_csr:
        return _wrap(torch.sparse_csr_tensor(t.crow_indices(), t.col_indices(), fn(t.values()), t.shape))
    return _wrap(fn(t))


def relu(x, name=None):
    return _vals(x, torch.relu)


def relu6(x, name=None):
    return _vals(x, lambda v: v.clamp(0, 6))


def leaky_relu(x, negative_slope=0.01, name=None):
    return _vals(x, lambda v: TF.leaky_relu(v, negative_slope))


def softmax(x, axis=-1, name=None):
    """Row softmax over the stored entries of each row (CSR or COO), zeros excluded."""
    t = x._t
    if axis != -1:
        raise ValueError("sparse softmax supports axis=-1 only")
    csr = t.layout == torch.sparse_csr
    coo = (t.to_sparse_coo() if csr else t).coalesce()
    out = torch.sparse.softmax(coo, -1).coalesce()
    return _wrap(out.to_sparse_csr() if csr else out)


def _triple(v):
    return [v] * 3 if isinstance(v, int) else list(v)


def _coords_key(c, dims):
    # c: [n, 4] (b, z, y, x) -> unique int64 key
    D, H, W = dims
    return ((c[:, 0] * D + c[:, 1]) * H + c[:, 2]) * W + c[:, 3]


def _sparse_conv(x, weight, bias, stride, padding, dilation, subm):
    t = x._t.coalesce()
    w = weight._t  # [kd, kh, kw, cin, cout]
    idx = t.indices().t()  # [n, 4]
    feats = t.values()  # [n, cin]
    N, D, H, W, _ = t.shape
    k = list(w.shape[:3])
    s, p, d = _triple(stride), _triple(padding), _triple(dilation)
    if subm:
        s, out_dims = [1, 1, 1], [D, H, W]
        p = [(k[i] - 1) // 2 * d[i] for i in range(3)]
    else:
        out_dims = [(sz + 2 * p[i] - d[i] * (k[i] - 1) - 1) // s[i] + 1 for i, sz in enumerate((D, H, W))]
    cout = w.shape[-1]
    out_keys, pairs = None, []
    if subm:
        out_coords = idx
    else:
        cand = []
        for off in itertools.product(*[range(kk) for kk in k]):
            num = [idx[:, i + 1] + p[i] - off[i] * d[i] for i in range(3)]
            ok = torch.ones(idx.shape[0], dtype=torch.bool, device=idx.device)
            oc = []
            for i in range(3):
                ok &= (num[i] % s[i] == 0)
                o = num[i] // s[i]
                ok &= (o >= 0) & (o < out_dims[i])
                oc.append(o)
            cand.append(torch.stack([idx[:, 0]] + oc, 1)[ok])
        out_coords = torch.unique(torch.cat(cand, 0), dim=0) if cand else idx[:0]
    okey = _coords_key(out_coords, out_dims)
    order = torch.argsort(okey)
    okey_sorted = okey[order]
    out = torch.zeros(out_coords.shape[0], cout, dtype=feats.dtype, device=feats.device)
    for off in itertools.product(*[range(kk) for kk in k]):
        num = [idx[:, i + 1] + p[i] - off[i] * d[i] for i in range(3)]
        ok = torch.ones(idx.shape[0], dtype=torch.bool, device=idx.device)
        oc = []
        for i in range(3):
            ok &= (num[i] % s[i] == 0)
            o = torch.div(num[i], s[i], rounding_mode="floor")
            ok &= (o >= 0) & (o < out_dims[i])
            oc.append(o)
        src = ok.nonzero().squeeze(1)
        if src.numel() == 0:
            continue
        key = _coords_key(torch.stack([idx[src, 0]] + [o[src] for o in oc], 1), out_dims)
        pos = torch.searchsorted(okey_sorted, key).clamp_max(max(okey_sorted.numel() - 1, 0))
        hit = okey_sorted[pos] == key
        if not bool(hit.any()):
            continue
        dst = order[pos[hit]]
        contrib = feats[src[hit]] @ w[off[0], off[1], off[2]]  # gather-GEMM
        out.index_add_(0, dst, contrib)  # scatter
    if bias is not None:
        out = out + bias._t
    return _wrap(torch.sparse_coo_tensor(out_coords.t(), out, (N, *out_dims, cout)).coalesce())


def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NDHWC", name=None):
    return _sparse_conv(x, weight, bias, stride, padding, dilation, subm=False)


def subm_conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NDHWC", key=None,
                name=None):
    return _sparse_conv(x, weight, bias, stride, padding, dilation, subm=True)


def max_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, data_format="NDHWC", name=None):
    """Max over the active sites in each window (inactive sites do not contribute)."""
    t = x._t.coalesce()
    idx = t.indices().t()
    feats = t.values()
    N, D, H, W, C = t.shape
    k = _triple(kernel_size)
    s = _triple(stride if stride is not None else kernel_size)
    p = _triple(padding)
    out_dims = [(sz + 2 * p[i] - k[i]) // s[i] + 1 for i, sz in enumerate((D, H, W))]
    keys, rows, dsts = [], [], []
    for off in itertools.product(*[range(kk) for kk in k]):
        num = [idx[:, i + 1] + p[i] - off[i] for i in range(3)]
        ok = torch.ones(idx.shape[0], dtype=torch.bool, device=idx.device)
        oc = []
        for i in range(3):
            ok &= (num[i] % s[i] == 0)
            o = torch.div(num[i], s[i], rounding_mode="floor")
            ok &= (o >= 0) & (o < out_dims[i])
            oc.append(o)
        src = ok.nonzero().squeeze(1)
        keys.append(torch.stack([idx[src, 0]] + [o[src] for o in oc], 1))
        rows.append(src)
    allc = torch.cat(keys, 0)
    allr = torch.cat(rows, 0)
    uniq, inv = torch.unique(allc, dim=0, return_inverse=True)
    out = torch.full((uniq.shape[0], C), float("-inf"), dtype=feats.dtype, device=feats.device)
    out = out.scatter_reduce(0, inv.unsqueeze(1).expand(-1, C), feats[allr], reduce="amax", include_self=True)
    return _wrap(torch.sparse_coo_tensor(uniq.t(), out, (N, *out_dims, C)).coalesce())


def attention(query, key, value, sparse_mask, key_padding_mask=None, attn_mask=None, name=None):
    """softmax(QK^T/sqrt(d) restricted to sparse_mask's pattern) @ V (reference transformer.py:22).
    query/key/value: [B, H, S, D] dense; sparse_mask: CSR [B*H, S, S]."""
    q, k, v = query._t, key._t, value._t
    B, Hh, S, Dd = q.shape
    m = sparse_mask._t
    dense_mask = (m.to_dense() if m.layout != torch.strided else m).reshape(B, Hh, S, S) != 0
    scores = (q @ k.transpose(-1, -2)) / (Dd ** 0.5)
    if key_padding_mask is not None:
        dense_mask = dense_mask & (key_padding_mask._t.reshape(B, 1, 1, S) != 0)
    if attn_mask is not None:
        dense_mask = dense_mask & (attn_mask._t.reshape(1, 1, S, S) != 0)
    scores = scores.masked_fill(~dense_mask, float("-inf"))
    probs = torch.softmax(scores, -1).nan_to_num(0.0)
    return _wrap(probs @ v)
