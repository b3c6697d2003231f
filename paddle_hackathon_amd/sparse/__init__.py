"""``paddle.sparse`` — COO/CSR sparse tensors (reference: python/paddle/incubate/sparse/
{creation,unary,binary,multiary}.py). Storage and kernels are torch sparse layouts, which
run on hipSPARSE on the MI355X. Unary ops act on the stored values only (zeros stay zero),
matching the reference's sparse kernels."""
from __future__ import annotations

import math
import warnings

import numpy as np
import torch

from ..framework.core import Tensor, _wrap, _unwrap, convert_dtype, _to_torch_device, default_device
from . import nn  # noqa: F401

warnings.filterwarnings("ignore", message="Sparse CSR tensor support is in beta")

__all__ = ["sparse_coo_tensor", "sparse_csr_tensor", "sin", "tan", "asin", "atan", "sinh", "tanh", "asinh", "atanh",
           "sqrt", "square", "log1p", "abs", "pow", "cast", "neg", "deg2rad", "rad2deg", "expm1", "mv", "matmul",
           "masked_matmul", "addmm", "add", "subtract", "multiply", "divide", "coalesce"]


def _arr(x, dtype=None, device=None):
    if isinstance(x, Tensor):
        t = x._t
    elif isinstance(x, torch.Tensor):
        t = x
    else:
        t = torch.as_tensor(np.asarray(x))
    if dtype is not None:
        t = t.to(convert_dtype(dtype))
    return t.to(device) if device is not None else t


def sparse_coo_tensor(indices, values, shape=None, dtype=None, place=None, stop_gradient=True):
    dev = _to_torch_device(place) if place is not None else default_device()
    idx = _arr(indices, device=dev).long()
    val = _arr(values, dtype, dev)
    if val.dtype == torch.float64 and dtype is None and not isinstance(values, (Tensor, torch.Tensor)):
        val = val.float()
    if shape is None:
        shape = (idx.max(1).values + 1).tolist() + list(val.shape[1:])
    t = torch.sparse_coo_tensor(idx, val, size=tuple(shape), device=dev)
    out = _wrap(t)
    out.stop_gradient = stop_gradient
    return out


def sparse_csr_tensor(crows, cols, values, shape, dtype=None, place=None, stop_gradient=True):
    dev = _to_torch_device(place) if place is not None else default_device()
    val = _arr(values, dtype, dev)
    if val.dtype == torch.float64 and dtype is None and not isinstance(values, (Tensor, torch.Tensor)):
        val = val.float()
    t = torch.sparse_csr_tensor(_arr(crows, device=dev).long(), _arr(cols, device=dev).long(), val,
                                size=tuple(shape), device=dev)
    out = _wrap(t)
    out.stop_gradient = stop_gradient
    return out


def _map_values(x, fn):
    t = _unwrap(x)
    if t.is_sparse:
        c = t.coalesce()
        return _wrap(torch.sparse_coo_tensor(c.indices(), fn(c.values()), c.shape, is_coalesced=True))
    if t.layout == torch.sparse_csr:
        return _wrap(torch.sparse_csr_tensor(t.crow_indices(), t.col_indices(), fn(t.values()), t.shape))
    return _wrap(fn(t))


def _unary(fn):
    def op(x, name=None):
        return _map_values(x, fn)
    return op


sin, tan, asin, atan, sinh, tanh, asinh, atanh = (_unary(f) for f in (torch.sin, torch.tan, torch.asin, torch.atan,
                                                                       torch.sinh, torch.tanh, torch.asinh,
                                                                       torch.atanh))
sqrt, square, log1p, abs, neg, expm1 = (_unary(f) for f in (torch.sqrt, torch.square, torch.log1p, torch.abs,
                                                            torch.neg, torch.expm1))
deg2rad = _unary(lambda v: v * (math.pi / 180.0))
rad2deg = _unary(lambda v: v * (180.0 / math.pi))


def pow(x, factor, name=None):
    return _map_values(x, lambda v: v.pow(factor))


def cast(x, index_dtype=None, value_dtype=None, name=None):
    t = _unwrap(x)
    vd = convert_dtype(value_dtype) if value_dtype else None
    idt = convert_dtype(index_dtype) if index_dtype else None
    if t.is_sparse:
        c = t.coalesce()
        v = c.values().to(vd) if vd else c.values()
        # torch keeps COO indices int64; the requested index dtype is recorded for parity only
        out = _wrap(torch.sparse_coo_tensor(c.indices(), v, c.shape, is_coalesced=True))
    else:
        v = t.values().to(vd) if vd else t.values()
        out = _wrap(torch.sparse_csr_tensor(t.crow_indices().to(idt or torch.int64), t.col_indices().to(idt or torch.int64),
                                            v, t.shape))
    return out


def coalesce(x):
    return _wrap(_unwrap(x).coalesce())


def _sp_or_dense(t):
    return t


def matmul(x, y, name=None):
    a, b = _unwrap(x), _unwrap(y)
    if a.layout == torch.sparse_csr and b.layout == torch.sparse_csr:
        return _wrap(torch.sparse.mm(a.to_sparse_coo(), b.to_sparse_coo()).to_sparse_csr())
    if a.is_sparse and b.is_sparse:
        return _wrap(torch.sparse.mm(a, b))
    if a.layout == torch.sparse_csr or a.is_sparse:
        if a.dim() == 3:
            return _wrap(torch.stack([torch.sparse.mm(a[i] if a.is_sparse else a.to_dense()[i].to_sparse(), b[i])
                                      for i in range(a.shape[0])]))
        return _wrap(torch.sparse.mm(a, b))
    return _wrap(torch.matmul(a, b))


def masked_matmul(x, y, mask, name=None):
    """dense x @ dense y, evaluated only at the non-zeros of sparse ``mask`` (SDDMM)."""
    a, b, m = _unwrap(x), _unwrap(y), _unwrap(mask)
    if m.layout == torch.sparse_csr:
        return _wrap(torch.sparse.sampled_addmm(m, a, b, beta=0.0, alpha=1.0) if a.dim() == 2 else
                     _sddmm_coo(a, b, m.to_sparse_coo()).to_sparse_csr())
    return _wrap(_sddmm_coo(a, b, m))


def _sddmm_coo(a, b, m):
    c = m.coalesce()
    idx = c.indices()
    if a.dim() == 2:
        vals = (a[idx[0]] * b[:, idx[1]].t()).sum(-1)
    else:
        vals = (a[idx[0], idx[1]] * b[idx[0], :, idx[2]]).sum(-1)
    return torch.sparse_coo_tensor(idx, vals, c.shape)


def mv(x, vec, name=None):
    a, v = _unwrap(x), _unwrap(vec)
    return _wrap(torch.mv(a if a.is_sparse else a.to_sparse_coo(), v) if a.layout != torch.sparse_csr
                 else torch.mv(a, v))


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):
    i, a, b = _unwrap(input), _unwrap(x), _unwrap(y)
    prod = _unwrap(matmul(_wrap(a), _wrap(b)))
    if i.is_sparse or i.layout == torch.sparse_csr:
        if prod.is_sparse or prod.layout == torch.sparse_csr:
            res = (beta * i.to_dense() + alpha * prod.to_dense())
            return _wrap(res.to_sparse_csr() if i.layout == torch.sparse_csr else res.to_sparse())
        return _wrap(beta * i.to_dense() + alpha * prod)
    return _wrap(beta * i + alpha * (prod.to_dense() if prod.is_sparse or prod.layout == torch.sparse_csr else prod))


def _binary(fn):
    def op(x, y, name=None):
        a, b = _unwrap(x), _unwrap(y)
        csr = a.layout == torch.sparse_csr
        if csr:
            a, b = a.to_sparse_coo(), b.to_sparse_coo() if b.layout == torch.sparse_csr else b
        if a.is_sparse and b.is_sparse:
            # same sparsity pattern union: operate on dense then re-sparsify over the union
            a, b = a.coalesce(), b.coalesce()
            union = torch.sparse_coo_tensor(torch.cat([a.indices(), b.indices()], 1),
                                            torch.ones(a._nnz() + b._nnz(), device=a.device), a.shape).coalesce()
            idx = union.indices()
            da, db = a.to_dense(), b.to_dense()
            vals = fn(da[tuple(idx)], db[tuple(idx)])
            out = torch.sparse_coo_tensor(idx, vals, a.shape).coalesce()
        else:
            out = fn(a.to_dense() if a.is_sparse else a, b.to_dense() if b.is_sparse else b)
        if csr:
            out = out.to_sparse_csr() if out.is_sparse else out
        return _wrap(out)
    return op


add = _binary(torch.add)
subtract = _binary(torch.sub)
multiply = _binary(torch.mul)
divide = _binary(torch.div)

for _n in __all__:
    if _n in globals() and callable(globals()[_n]) and getattr(globals()[_n], "__name__", "") in ("op", "<lambda>"):
        globals()[_n].__name__ = _n
