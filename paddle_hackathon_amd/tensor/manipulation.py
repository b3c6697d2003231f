"""Shape / layout manipulation ops (reference: python/paddle/tensor/manipulation.py)."""
from __future__ import annotations

import numpy as np
import torch

from ..framework.core import Tensor, convert_dtype
from ..framework.dispatch import register_ops
from ._helpers import _u, _w, _axis, _int_list

__all__ = [
    "cast", "concat", "broadcast_tensors", "expand", "broadcast_to", "expand_as", "tile",
    "flatten", "flatten_", "gather", "gather_nd", "reshape", "reshape_", "reverse", "flip",
    "scatter", "scatter_", "scatter_nd_add", "scatter_nd", "shard_index", "slice", "crop",
    "split", "squeeze", "squeeze_", "stack", "strided_slice", "unique", "unique_consecutive",
    "unsqueeze", "unsqueeze_", "unstack", "rot90", "unbind", "roll", "chunk", "tolist",
    "take_along_axis", "put_along_axis", "put_along_axis_", "tensordot", "as_complex",
    "as_real", "moveaxis", "repeat_interleave", "transpose", "t", "index_select",
    "masked_select", "index_sample", "where", "nonzero", "index_add", "index_put",
    "view", "view_as", "vsplit", "hsplit", "dsplit", "atleast_1d", "atleast_2d", "atleast_3d",
    "masked_fill", "fill_", "zero_", "fill_diagonal_", "unfold", "expand_", "one_hot_index",
]


def cast(x, dtype):
    return _w(_u(x).to(convert_dtype(dtype)))


def _paddle_shape(t, shape):
    shape = _int_list(shape)
    # paddle: 0 means copy the corresponding input dim
    if any(s == 0 for s in shape):
        shape = [t.shape[i] if s == 0 else s for i, s in enumerate(shape)]
    return shape


def reshape(x, shape, name=None):
    t = x._t
    return _w(t.reshape(_paddle_shape(t, shape)))


def reshape_(x, shape, name=None):
    x._t = x._t.reshape(_paddle_shape(x._t, shape))
    return x


def view(x, shape_or_dtype, name=None):
    if isinstance(shape_or_dtype, (list, tuple, Tensor)):
        return _w(x._t.view(_paddle_shape(x._t, shape_or_dtype)))
    return _w(x._t.view(convert_dtype(shape_or_dtype)))


def view_as(x, other, name=None):
    return _w(x._t.view_as(_u(other)))


def transpose(x, perm, name=None):
    return _w(_u(x).permute(*_int_list(perm)))


def t(input, name=None):
    tt = _u(input)
    if tt.dim() < 2:
        return _w(tt)
    return _w(tt.t())


def moveaxis(x, source, destination, name=None):
    return _w(torch.movedim(_u(x), source, destination))


def concat(x, axis=0, name=None):
    if isinstance(axis, Tensor):
        axis = int(axis._t.item())
    return _w(torch.cat([_u(v) for v in x], dim=axis))


def stack(x, axis=0, name=None):
    return _w(torch.stack([_u(v) for v in x], dim=axis))


def _sections(t, num_or_sections, axis):
    n = t.shape[axis]
    if isinstance(num_or_sections, (int, np.integer)):
        if n % num_or_sections != 0:
            raise ValueError(f"split: dim {n} not divisible by {num_or_sections}")
        return [n // num_or_sections] * int(num_or_sections)
    secs = _int_list(num_or_sections)
    if -1 in secs:
        i = secs.index(-1)
        secs[i] = n - (sum(secs) + 1)
    return secs


def split(x, num_or_sections, axis=0, name=None):
    t = _u(x)
    if isinstance(axis, Tensor):
        axis = int(axis._t.item())
    axis = axis % t.dim()
    return [_w(p) for p in torch.split(t, _sections(t, num_or_sections, axis), dim=axis)]


def vsplit(x, num_or_sections, name=None):
    return split(x, num_or_sections, 0)


def hsplit(x, num_or_sections, name=None):
    return split(x, num_or_sections, 1)


def dsplit(x, num_or_sections, name=None):
    return split(x, num_or_sections, 2)


def chunk(x, chunks, axis=0, name=None):
    return split(x, chunks, axis)


def unbind(input, axis=0):
    return [_w(p) for p in torch.unbind(_u(input), axis)]


def unstack(x, axis=0, num=None):
    return [_w(p) for p in torch.unbind(_u(x), axis)]


def squeeze(x, axis=None, name=None):
    tt = _u(x)
    if axis is None:
        return _w(tt.squeeze())
    axes = _int_list(axis)
    axes = [a % tt.dim() for a in axes if tt.shape[a] == 1] if tt.dim() else []
    if not axes:
        return _w(tt)
    return _w(tt.squeeze(tuple(axes)))


def squeeze_(x, axis=None, name=None):
    x._t = squeeze(x, axis)._t
    return x


def unsqueeze(x, axis, name=None):
    tt = _u(x)
    axes = _int_list(axis)
    for a in axes:
        a = a if a >= 0 else a + tt.dim() + 1
        tt = tt.unsqueeze(a)
    return _w(tt)


def unsqueeze_(x, axis, name=None):
    x._t = unsqueeze(x, axis)._t
    return x


def flatten(x, start_axis=0, stop_axis=-1, name=None):
    tt = _u(x)
    if tt.dim() == 0:
        return _w(tt.reshape(1))
    return _w(torch.flatten(tt, start_axis, stop_axis))


def flatten_(x, start_axis=0, stop_axis=-1, name=None):
    x._t = flatten(x, start_axis, stop_axis)._t
    return x


def expand(x, shape, name=None):
    tt = _u(x)
    shape = _int_list(shape)
    return _w(tt.expand(*shape))


expand_ = expand


def broadcast_to(x, shape, name=None):
    return expand(x, shape)


def expand_as(x, y, name=None):
    return _w(_u(x).expand_as(_u(y)))


def broadcast_tensors(input, name=None):
    return [_w(p) for p in torch.broadcast_tensors(*[_u(v) for v in input])]


def tile(x, repeat_times, name=None):
    return _w(_u(x).repeat(*_pad_reps(_u(x), _int_list(repeat_times))))


def _pad_reps(tt, reps):
    if len(reps) < tt.dim():
        reps = [1] * (tt.dim() - len(reps)) + reps
    return reps


def flip(x, axis, name=None):
    return _w(torch.flip(_u(x), _int_list(axis)))


reverse = flip


def rot90(x, k=1, axes=[0, 1], name=None):
    return _w(torch.rot90(_u(x), k, axes))


def roll(x, shifts, axis=None, name=None):
    tt = _u(x)
    shifts = _int_list(shifts)
    if axis is None:
        return _w(torch.roll(tt, shifts))
    return _w(torch.roll(tt, shifts, _int_list(axis)))


def gather(x, index, axis=None, name=None):
    tt = _u(x)
    idx = _u(index)
    if axis is None:
        axis = 0
    if isinstance(axis, Tensor):
        axis = int(axis._t.item())
    if idx.dim() == 0:
        return _w(tt.index_select(axis, idx.reshape(1)).squeeze(axis))
    return _w(tt.index_select(axis, idx.reshape(-1).long()))


def index_select(x, index, axis=0, name=None):
    return _w(torch.index_select(_u(x), axis, _u(index).long()))


def gather_nd(x, index, name=None):
    tt = _u(x)
    idx = _u(index).long()
    k = idx.shape[-1]
    flat = idx.reshape(-1, k)
    out = tt[tuple(flat[:, i] for i in range(k))]
    return _w(out.reshape(list(idx.shape[:-1]) + list(tt.shape[k:])))


def scatter(x, index, updates, overwrite=True, name=None):
    tt = _u(x)
    idx = _u(index).reshape(-1).long()
    up = _u(updates)
    if overwrite:
        return _w(tt.index_copy(0, idx, up) if idx.unique().numel() == idx.numel() else _scatter_last(tt, idx, up))
    out = tt.index_fill(0, idx, 0)
    return _w(out.index_add(0, idx, up))


def _scatter_last(tt, idx, up):
    out = tt.clone()
    out[idx] = up
    return out


def scatter_(x, index, updates, overwrite=True, name=None):
    x._t = scatter(x, index, updates, overwrite)._t
    return x


def scatter_nd_add(x, index, updates, name=None):
    tt = _u(x)
    idx = _u(index).long()
    k = idx.shape[-1]
    flat = idx.reshape(-1, k)
    up = _u(updates).reshape([flat.shape[0]] + list(tt.shape[k:]))
    out = tt.clone()
    out.index_put_(tuple(flat[:, i] for i in range(k)), up, accumulate=True)
    return _w(out)


def scatter_nd(index, updates, shape, name=None):
    up = _u(updates)
    z = torch.zeros(_int_list(shape), dtype=up.dtype, device=up.device)
    return scatter_nd_add(_w(z), index, updates)


def index_add(x, index, axis, value, name=None):
    return _w(_u(x).index_add(axis, _u(index).long(), _u(value)))


def index_put(x, indices, value, accumulate=False, name=None):
    return _w(_u(x).index_put(tuple(_u(i) for i in indices), _u(value), accumulate))


def shard_index(input, index_num, nshards, shard_id, ignore_value=-1):
    tt = _u(input)
    size = (index_num + nshards - 1) // nshards
    lo = shard_id * size
    inside = (tt >= lo) & (tt < lo + size)
    return _w(torch.where(inside, tt - lo, torch.full_like(tt, ignore_value)))


def slice(input, axes, starts, ends):
    tt = _u(input)
    idx = [builtins_slice(None)] * tt.dim()
    starts, ends = _int_list(starts), _int_list(ends)
    for a, s, e in zip(_int_list(axes), starts, ends):
        n = tt.shape[a]
        s = max(min(s + n if s < 0 else s, n), 0)
        e = max(min(e + n if e < 0 else e, n), 0)
        idx[a] = builtins_slice(s, e)
    return _w(tt[tuple(idx)])


import builtins as _b  # noqa: E402

builtins_slice = _b.slice


def strided_slice(x, axes, starts, ends, strides, name=None):
    tt = _u(x)
    idx = [builtins_slice(None)] * tt.dim()
    for a, s, e, st in zip(_int_list(axes), _int_list(starts), _int_list(ends), _int_list(strides)):
        n = tt.shape[a]
        if st > 0:
            s = max(min(s + n if s < 0 else s, n), 0)
            e = max(min(e + n if e < 0 else e, n), 0)
            idx[a] = builtins_slice(s, e, st)
        else:
            # negative stride: flip then slice
            s = s + n if s < 0 else min(s, n - 1)
            e = e + n if e < 0 else e
            sel = torch.arange(s, max(e, -1), st, device=tt.device)
            sel = sel[(sel >= 0) & (sel < n)]
            tt = tt.index_select(a, sel)
    return _w(tt[tuple(idx)])


def crop(x, shape=None, offsets=None, name=None):
    tt = _u(x)
    shape = _int_list(shape) if shape is not None else list(tt.shape)
    offsets = _int_list(offsets) if offsets is not None else [0] * tt.dim()
    idx = tuple(builtins_slice(o, o + (s if s != -1 else tt.shape[i] - o)) for i, (o, s) in enumerate(zip(offsets, shape)))
    return _w(tt[idx])


def unique(x, return_index=False, return_inverse=False, return_counts=False, axis=None, dtype="int64", name=None):
    tt = _u(x)
    dt = convert_dtype(dtype)
    if axis is None:
        flat = tt.reshape(-1)
        out, inv, cnt = torch.unique(flat, sorted=True, return_inverse=True, return_counts=True)
    else:
        out, inv, cnt = torch.unique(tt, sorted=True, return_inverse=True, return_counts=True, dim=axis)
        flat = None
    res = [_w(out)]
    if return_index:
        n = inv.numel()
        first = torch.full((out.shape[0] if axis is not None else out.numel(),), n, dtype=torch.int64, device=tt.device)
        first.scatter_reduce_(0, inv.reshape(-1), torch.arange(n, device=tt.device), reduce="amin")
        res.append(_w(first.to(dt)))
    if return_inverse:
        res.append(_w(inv.to(dt)))
    if return_counts:
        res.append(_w(cnt.to(dt)))
    return res[0] if len(res) == 1 else tuple(res)


def unique_consecutive(x, return_inverse=False, return_counts=False, axis=None, dtype="int64", name=None):
    out, inv, cnt = torch.unique_consecutive(_u(x), return_inverse=True, return_counts=True, dim=axis)
    res = [_w(out)]
    if return_inverse:
        res.append(_w(inv.to(convert_dtype(dtype))))
    if return_counts:
        res.append(_w(cnt.to(convert_dtype(dtype))))
    return res[0] if len(res) == 1 else tuple(res)


def tolist(x):
    return _u(x).tolist()


def take_along_axis(arr, indices, axis):
    a, i = _u(arr), _u(indices).long()
    if a.dim() == i.dim():
        shape = list(torch.broadcast_shapes(*[tuple(s if d != axis % a.dim() else 1 for d, s in enumerate(t.shape)) for t in (a, i)]))
        ishape = list(shape)
        ishape[axis % a.dim()] = i.shape[axis]
        ashape = list(shape)
        ashape[axis % a.dim()] = a.shape[axis]
        a = a.expand(ashape)
        i = i.expand(ishape)
    return _w(torch.gather(a, axis, i))


def put_along_axis(arr, indices, values, axis, reduce="assign"):
    a, i = _u(arr), _u(indices).long()
    v = _u(values)
    if not isinstance(v, torch.Tensor):
        v = torch.full(i.shape, v, dtype=a.dtype, device=a.device)
    v = v.expand(i.shape) if v.shape != i.shape else v
    if reduce == "assign":
        return _w(a.scatter(axis, i, v))
    red = {"add": "sum", "multiply": "prod", "mul": "prod"}[reduce]
    return _w(a.scatter_reduce(axis, i, v, reduce=red))


def put_along_axis_(arr, indices, values, axis, reduce="assign"):
    arr._t = put_along_axis(arr, indices, values, axis, reduce)._t
    return arr


def tensordot(x, y, axes=2, name=None):
    if isinstance(axes, Tensor):
        axes = axes._t.tolist()
    return _w(torch.tensordot(_u(x), _u(y), dims=axes))


def as_complex(x, name=None):
    return _w(torch.view_as_complex(_u(x).contiguous()))


def as_real(x, name=None):
    return _w(torch.view_as_real(_u(x)))


def repeat_interleave(x, repeats, axis=None, name=None):
    r = _u(repeats)
    return _w(torch.repeat_interleave(_u(x), r, dim=axis))


def masked_select(x, mask, name=None):
    return _w(torch.masked_select(_u(x), _u(mask)))


def masked_fill(x, mask, value, name=None):
    v = value._t if isinstance(value, Tensor) else value
    return _w(_u(x).masked_fill(_u(mask), v))


def index_sample(x, index):
    return _w(torch.gather(_u(x), 1, _u(index).long()))


def where(condition, x=None, y=None, name=None):
    c = _u(condition)
    if x is None and y is None:
        return nonzero(condition, as_tuple=True)
    xt = _u(x)
    yt = _u(y)
    if not isinstance(xt, torch.Tensor):
        xt = torch.as_tensor(xt, dtype=yt.dtype if isinstance(yt, torch.Tensor) else None, device=c.device)
    if not isinstance(yt, torch.Tensor):
        yt = torch.as_tensor(yt, dtype=xt.dtype, device=c.device)
    return _w(torch.where(c.bool(), xt, yt))


def nonzero(x, as_tuple=False):
    tt = _u(x)
    if as_tuple:
        return tuple(_w(v.unsqueeze(-1)) for v in torch.nonzero(tt, as_tuple=True))
    return _w(torch.nonzero(tt))


def atleast_1d(*inputs, name=None):
    r = [_w(torch.atleast_1d(_u(v))) for v in inputs]
    return r[0] if len(r) == 1 else r


def atleast_2d(*inputs, name=None):
    r = [_w(torch.atleast_2d(_u(v))) for v in inputs]
    return r[0] if len(r) == 1 else r


def atleast_3d(*inputs, name=None):
    r = [_w(torch.atleast_3d(_u(v))) for v in inputs]
    return r[0] if len(r) == 1 else r


def fill_(x, value):
    with torch.no_grad():
        x._t.fill_(value)
    return x


def zero_(x):
    with torch.no_grad():
        x._t.zero_()
    return x


def fill_diagonal_(x, value, offset=0, wrap=False, name=None):
    with torch.no_grad():
        if offset == 0:
            x._t.fill_diagonal_(value, wrap)
        else:
            d = torch.diagonal(x._t, offset)
            d.fill_(value)
    return x


def unfold(x, axis, size, step, name=None):
    return _w(_u(x).unfold(axis, size, step))


def one_hot_index(x, num_classes):
    return _w(torch.nn.functional.one_hot(_u(x).long(), num_classes))


register_ops(globals(), __all__)
