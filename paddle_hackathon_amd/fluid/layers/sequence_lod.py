"""``fluid.layers`` sequence (LoD) ops (reference: python/paddle/fluid/layers/sequence_lod.py;
kernels paddle/fluid/operators/sequence_ops/*). Inputs are LoD tensors (flat [sum(len), ...]
rows with a ``_lod`` offset table, see fluid/core.py); each op pads to [B, Tmax, ...], computes
with length masks, and returns LoD rows again. Padded tensors plus explicit lengths work too.

Static Programs. Every op records ONE op (``sequence_pool`` ... typed by the reference op name in a
saved ProgramDesc, static/ref_emit.py) whose LoD is resolved when the Executor runs it: fed LoD
tensors keep their offsets, ops that keep the row count share their input's LoD (the reference's
ShareLoD, static/program.py run_block), and the sequence ops read / write the offsets at run
time. At build time (meta tensors, no LoD yet) a LoD input is taken as one sequence, which gives
the outputs their static shapes (batch dim 1 = the -1 of the declared shape).
``sequence_conv`` creates its filter at build time and records the pure ``sequence_conv_op``."""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from ._common import T, W, dev, to_padded, from_padded, mask_of, register
from .. import core as fcore

__all__ = ["sequence_conv", "sequence_softmax", "sequence_pool", "sequence_concat", "sequence_first_step",
           "sequence_last_step", "sequence_slice", "sequence_expand", "sequence_expand_as", "sequence_pad",
           "sequence_unpad", "sequence_reshape", "sequence_scatter", "sequence_enumerate", "sequence_mask",
           "sequence_reverse"]


def _lod(x):
    return fcore.lod_of(x)


def _meta(x):
    return T(x).device.type == "meta"


def _seq_offsets(x):
    lod = _lod(x)
    if not lod:
        if _meta(x):                       # build time: one sequence of all rows
            return [0, T(x).shape[0]]
        raise ValueError("sequence op: input has no LoD (build it with fluid.create_lod_tensor or set _lod)")
    return lod[-1]


def _padded(x):
    """(padded [B, Tmax, ...], lengths, had_lod); a build-time (meta) LoD input is one sequence"""
    if not _lod(x) and _meta(x):
        t = T(x)
        return t[None], torch.full((1,), t.shape[0], dtype=torch.long, device=t.device), True
    return to_padded(x)


def _out(t, lens, like):
    o = W(t)
    o._lod = _lod(like)[:-1] + [fcore._offsets_from_lengths(lens)]
    return o


def sequence_conv(input, num_filters, filter_size=3, filter_stride=1, padding=True, padding_start=None,
                  bias_attr=None, param_attr=None, act=None, name=None):
    """context projection of ``filter_size`` rows starting at ``padding_start`` (default
    -(filter_size // 2)), zero outside each sequence, times a [filter_size * D, num_filters]
    filter (sequence_conv_op.h)"""
    from ._common import fparam as _create_parameter
    from ._common import act as _act
    D = T(input).shape[1]
    w = _create_parameter([filter_size * D, num_filters], T(input).dtype, param_attr)
    b = _create_parameter([num_filters], T(input).dtype, bias_attr, is_bias=True) if bias_attr is not False else None
    start = -(filter_size // 2) if padding_start is None else padding_start
    conv = sequence_conv_op(input, w, None, filter_size, start, filter_stride)
    out = conv
    if b is not None:   # the bias is its own elementwise_add op, as in the reference builder
        from ...tensor import math as _m
        out = _m.add(out, b)
    out = _act(out, act)
    if out is not conv and _lod(conv):   # dygraph: the elementwise ops keep the rows (ShareLoD)
        out._lod = _lod(conv)
    return out


def sequence_conv_op(input, filter, bias=None, context_length=3, context_start=-1, context_stride=1):
    """the recorded sequence_conv op (Input, Filter [, Bias]; contextLength / contextStart /
    contextStride)"""
    p, lens, _ = _padded(input)
    Tm = p.shape[1]
    m = mask_of(lens, Tm, p.device)
    p = p * m[..., None]
    cols = []
    for k in range(context_length):
        s = context_start + k
        sh = torch.zeros_like(p)
        if s >= 0:
            sh[:, :Tm - s] = p[:, s:] if s < Tm else sh[:, :0]
        else:
            sh[:, -s:] = p[:, :Tm + s] if -s < Tm else sh[:, :0]
        cols.append(sh)
    y = torch.cat(cols, -1) @ T(filter)
    if bias is not None:
        y = y + T(bias)
    return from_padded(y, lens, _lod(input))


def sequence_softmax(input, use_cudnn=False, name=None):
    p, lens, _ = _padded(input)
    v = p.reshape(p.shape[0], p.shape[1])
    m = mask_of(lens, v.shape[1], v.device)
    s = torch.softmax(v.masked_fill(~m, float("-inf")), 1).nan_to_num(0.0)
    return from_padded(s[..., None], lens, _lod(input))


def sequence_pool(input, pool_type, is_test=False, pad_value=0.0):
    """sum / average / sqrt / max / last / first per sequence -> [B, D]; empty sequences give
    ``pad_value``"""
    p, lens, _ = _padded(input)
    B, Tm = p.shape[:2]
    m = mask_of(lens, Tm, p.device)
    mf = m.reshape(B, Tm, *([1] * (p.dim() - 2))).to(p.dtype)
    pt = pool_type.lower()
    n = lens.clamp_min(1).to(p.dtype).reshape(B, *([1] * (p.dim() - 2)))
    if pt == "sum":
        r = (p * mf).sum(1)
    elif pt == "average":
        r = (p * mf).sum(1) / n
    elif pt == "sqrt":
        r = (p * mf).sum(1) / n.sqrt()
    elif pt == "max":
        r = p.masked_fill(mf == 0, float("-inf")).amax(1)
    elif pt == "first":
        r = p[:, 0]
    elif pt == "last":
        r = p[torch.arange(B, device=p.device), (lens - 1).clamp_min(0)]
    else:
        raise ValueError(f"sequence_pool: pool_type {pool_type!r}")
    empty = (lens == 0).reshape(B, *([1] * (r.dim() - 1)))
    out = W(torch.where(empty, torch.full_like(r, pad_value), r))
    if len(_lod(input)) > 1:              # a 2-level input keeps its outer level
        out._lod = _lod(input)[:-1]
    return out


def sequence_first_step(input):
    return sequence_pool(input, "first")


def sequence_last_step(input):
    return sequence_pool(input, "last")


def sequence_concat(input, name=None):
    """concatenate the i-th sequences of every input, for each i"""
    if not _lod(input[0]) and _meta(input[0]):
        return W(torch.cat([T(x) for x in input], 0))
    offs = [_seq_offsets(x) for x in input]
    ts = [T(x) for x in input]
    parts, lens = [], []
    for i in range(len(offs[0]) - 1):
        n = 0
        for t, o in zip(ts, offs):
            parts.append(t[o[i]:o[i + 1]])
            n += o[i + 1] - o[i]
        lens.append(n)
    return _out(torch.cat(parts, 0), lens, input[0])


def sequence_slice(input, offset, length, name=None):
    if not _lod(input) and _meta(input):
        return W(T(input).clone())
    off = _seq_offsets(input)
    t = T(input)
    so = T(offset).reshape(-1).tolist()
    sl = T(length).reshape(-1).tolist()
    parts = [t[off[i] + int(so[i]):off[i] + int(so[i]) + int(sl[i])] for i in range(len(off) - 1)]
    return _out(torch.cat(parts, 0), [int(v) for v in sl], input)


def sequence_expand(x, y, ref_level=-1, name=None):
    """repeat each sequence (or row) of ``x`` as many times as ``y``'s ``ref_level`` LoD says"""
    ylod = _lod(y)
    t = T(x)
    if not ylod:
        if _meta(y) or _meta(x):           # build time: the output has x's row layout
            return W(t.clone())
        raise ValueError("sequence_expand: y has no LoD")
    ref = ylod[ref_level]
    reps = fcore._lengths_from_offsets(ref)
    xoff = _lod(x)[0] if _lod(x) else list(range(t.shape[0] + 1))
    parts, lens = [], []
    for i, r in enumerate(reps):
        seg = t[xoff[i]:xoff[i + 1]]
        for _ in range(r):
            parts.append(seg)
            lens.append(seg.shape[0])
    out = W(torch.cat(parts, 0) if parts else t[:0])
    out._lod = [fcore._offsets_from_lengths(lens)]
    return out


def sequence_expand_as(x, y, name=None):
    """row i of ``x`` repeated to the length of ``y``'s i-th sequence"""
    t = T(x)
    if not _lod(y) and _meta(y):
        return W(t.expand(T(y).shape[0], *t.shape[1:]).clone() if t.shape[0] == 1 else t.clone())
    lens = fcore._lengths_from_offsets(_seq_offsets(y))
    out = W(torch.repeat_interleave(t, torch.tensor(lens, device=t.device), 0))
    out._lod = [fcore._offsets_from_lengths(lens)]
    return out


def sequence_pad(x, pad_value, maxlen=None, name=None):
    """-> (padded [B, maxlen, ...], lengths [B] int64)"""
    p, lens, _ = _padded(x)
    pv = T(pad_value).reshape(-1)
    Tm = maxlen if maxlen is not None else p.shape[1]
    fill = pv.to(p.dtype).reshape(p.shape[2:]) if pv.numel() > 1 else pv.to(p.dtype).reshape(())
    out = fill.expand([p.shape[0], Tm] + list(p.shape[2:])).clone()
    n = min(Tm, p.shape[1])
    m = mask_of(lens, n, p.device).reshape(p.shape[0], n, *([1] * (p.dim() - 2)))
    out[:, :n] = torch.where(m, p[:, :n], out[:, :n])
    return W(out), W(lens.to(torch.int64))


def sequence_unpad(x, length, name=None):
    t = T(x)
    if _meta(x):
        return W(t.reshape(-1, *t.shape[2:]))
    lens = T(length).reshape(-1).long()
    return from_padded(t, lens)


def sequence_reshape(input, new_dim):
    t = T(input)
    if not _lod(input) and _meta(input):
        return W(t.reshape(-1, new_dim))
    D = t.shape[1]
    lens = [n * D // new_dim for n in fcore._lengths_from_offsets(_seq_offsets(input))]
    return _out(t.reshape(-1, new_dim), lens, input)


def sequence_scatter(input, index, updates, name=None):
    """out = input; out[i, index_j] += updates_j for the j-th row of the i-th update sequence"""
    t = T(input).clone()
    if _meta(input):
        return W(t)
    idx = T(index).reshape(-1).long()
    u = T(updates)
    uoff = _seq_offsets(updates)
    for i in range(len(uoff) - 1):
        a, b = uoff[i], uoff[i + 1]
        t[i].index_add_(0, idx[a:b], u[a:b].reshape(-1))
    return W(t)


def sequence_enumerate(input, win_size, pad_value=0, name=None):
    """every length-``win_size`` window starting at each position of each sequence (padded past
    the end)"""
    t = T(input).reshape(-1)
    if _meta(input):
        return W(t.new_zeros(t.shape[0], win_size))
    off = _seq_offsets(input)
    rows = []
    for i in range(len(off) - 1):
        seq = t[off[i]:off[i + 1]]
        for j in range(seq.shape[0]):
            w = seq[j:j + win_size]
            if w.shape[0] < win_size:
                w = torch.cat([w, torch.full((win_size - w.shape[0],), pad_value, dtype=t.dtype, device=t.device)])
            rows.append(w)
    out = W(torch.stack(rows) if rows else t.new_zeros(0, win_size))
    out._lod = _lod(input)
    return out


def sequence_mask(x, maxlen=None, dtype="int64", name=None):
    lens = T(x)
    if hasattr(maxlen, "_t"):
        m = 1 if _meta(maxlen) else int(T(maxlen).item())
    else:
        m = maxlen if maxlen is not None else (1 if lens.device.type == "meta" else int(lens.max()))
    r = torch.arange(m, device=lens.device)
    return W((r < lens[..., None]).to(fcore.convert_dtype(dtype)))


def sequence_reverse(x, name=None):
    t = T(x)
    if not _lod(x) and _meta(x):
        return W(t.flip(0))
    off = _seq_offsets(x)
    parts = [t[off[i]:off[i + 1]].flip(0) for i in range(len(off) - 1)]
    out = W(torch.cat(parts, 0))
    out._lod = _lod(x)
    return out


_ = (dev, TF)
# every op records one static op (sequence_conv records sequence_conv_op after creating its filter)
register(globals(), [n for n in __all__ if n != "sequence_conv"] + ["sequence_conv_op"])
