"""Shared helpers of the fluid layer functions: tensor unwrapping, in-place output writes that
work in both modes, fluid's axis broadcasting, and the LoD <-> padded conversions the sequence
layers use (reference: python/paddle/fluid/layer_helper.py, layers/nn.py _elementwise_op)."""
from __future__ import annotations

import numpy as np
import torch

from ...framework import core as _core
from ...framework.core import Tensor, _wrap, convert_dtype
from ...framework.dispatch import static_op, register_ops  # noqa: F401
from .. import core as fcore


def T(x):
    """-> torch tensor (Tensor, numpy, Python scalar / list)"""
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(np.asarray(x), device=_core.default_device())


def W(t, like=None):
    out = _wrap(t)
    if like is not None and fcore.lod_of(like):
        out._lod = fcore.lod_of(like)
    return out


def dev():
    return _core.default_device()


def dt(d):
    return fcore.convert_dtype(d) if d is not None else torch.float32


def is_static_var(x):
    from ...static.program import Variable
    return isinstance(x, Variable)


def static_mode():
    return _core._mode.static


def write_to(out, value):
    """store ``value`` into the existing tensor / Variable ``out`` (fluid ``out=``/``cond=``/in_place
    arguments). Static mode appends an ``assign`` op whose output IS ``out``, so readers of
    ``out`` after it (including later iterations of an enclosing While) see the new value;
    dynamic mode rebinds the storage of the handle."""
    if out is None:
        return value
    if static_mode() and (is_static_var(out) or is_static_var(value)):
        from ...static.program import OpDesc, default_main_program
        if is_static_var(out):
            op = OpDesc("assign", _identity, (value,), {}, out, attrs={"inplace_write": True})
        else:
            # a persistent (eager) tensor updated by the program: copy into its storage at run time
            def _copy_into(v, _dst=out):
                _dst._t = T(v).detach().to(_dst._t.dtype) if _dst._t.shape != T(v).shape else \
                    _dst._t.copy_(T(v).detach())
                return _dst
            op = OpDesc("assign", _copy_into, (value,), {}, [], attrs={"inplace_write": True, "persistent": out})
        default_main_program().current_block().append_op(op)
        return out
    v = T(value)
    if isinstance(out, Tensor):
        out._t = v.to(out._t.dtype) if out._t.dtype != v.dtype and out._t.numel() else v
        lod = fcore.lod_of(value)
        if lod:
            out._lod = lod
        return out
    return value


def _identity(x):
    return x


def act(x, name):
    if not name:
        return x
    from ...nn import functional as F
    return getattr(F, name)(x)


def bcast_y(xt, yt, axis):
    """fluid elementwise broadcasting: Y's dims align with X's starting at ``axis`` (-1: trailing)"""
    if axis is None or axis == -1 or yt.dim() >= xt.dim():
        return yt
    # trailing singleton dims of Y are trimmed (elementwise_op_function.h trim_trailing_singular_dims)
    shape = list(yt.shape)
    while len(shape) > 1 and shape[-1] == 1 and axis + len(shape) > xt.dim():
        shape.pop()
    post = xt.dim() - axis - len(shape)
    return yt.reshape([1] * axis + shape + [1] * max(post, 0))


def norm_axes(dim, nd):
    if dim is None:
        return list(range(nd))
    dims = dim if isinstance(dim, (list, tuple)) else [dim]
    return [d % nd if nd else 0 for d in dims]


# ----------------------------------------------------------------------------- LoD helpers
def level_offsets(x, level=-1):
    lod = fcore.lod_of(x)
    if not lod:
        return None
    return lod[level]


def to_padded(x, length=None, pad_value=0.0):
    """(padded [B, Tmax, ...], lengths LongTensor [B]) from a LoD tensor (last level) or from a
    padded tensor + ``length``"""
    t = T(x)
    off = level_offsets(x)
    if off is not None:
        lens = fcore._lengths_from_offsets(off)
        B, Tm = len(lens), max(lens) if lens else 0
        out = t.new_full([B, Tm] + list(t.shape[1:]), pad_value)
        for i, (a, n) in enumerate(zip(off[:-1], lens)):
            if n:
                out[i, :n] = t[a:a + n]
        return out, torch.tensor(lens, dtype=torch.long, device=t.device), True
    if length is None:
        lens = torch.full((t.shape[0],), t.shape[1], dtype=torch.long, device=t.device)
    else:
        lens = T(length).reshape(-1).long().to(t.device)
    return t, lens, False


def from_padded(p, lens, like_lod=None):
    """flat LoD tensor [sum(len), ...] from padded rows"""
    if lens.device.type == "meta" or p.device.type == "meta":   # static build: shapes only
        return _wrap(p.reshape(-1, *p.shape[2:]))
    ls = [int(n) for n in lens.tolist()]
    parts = [p[i, :n] for i, n in enumerate(ls)]
    flat = torch.cat(parts, 0) if parts else p.new_zeros([0] + list(p.shape[2:]))
    out = _wrap(flat)
    out._lod = (like_lod[:-1] if like_lod else []) + [fcore._offsets_from_lengths(ls)]
    return out


def mask_of(lens, Tm, device):
    return torch.arange(Tm, device=device)[None, :] < lens.to(device)[:, None]


def register(namespace, names, skip=()):
    """wrap every plain op function of a fluid layer module so a static-mode call records one op
    typed by its fluid name (parameter-creating and control-flow builders are skipped)"""
    register_ops(namespace, [n for n in names if n not in skip])


def _ensure_int_list(v, n):
    if isinstance(v, (list, tuple)):
        return [int(i) for i in v]
    return [int(v)] * n


__all__ = []
_ = convert_dtype


_NAMED_PARAMS = {}


def fparam(shape, dtype=None, attr=None, is_bias=False, default_initializer=None, name=None):
    """create a parameter for a fluid builder and remember it by name (get_parameter)"""
    from ...nn.layer.layers import _create_parameter
    p = _create_parameter(shape, dtype, attr, is_bias, default_initializer, name)
    if p is not None:
        _NAMED_PARAMS[p.name] = p
    return p


def static_source(fn, name, like):
    """static mode: record an input-free op (fill_constant, zeros ...) whose output Variable has
    ``like``'s shape / dtype, so later in-place writes (While bodies) can rebind it per run"""
    from ...static.program import OpDesc, Variable, default_main_program
    blk = default_main_program().current_block()
    v = Variable(blk, torch.empty(tuple(like.shape), dtype=like.dtype, device="meta"))
    blk.vars[v.name] = v
    op = OpDesc(name, fn, (), {}, v)
    v.op = op
    blk.append_op(op)
    return v
