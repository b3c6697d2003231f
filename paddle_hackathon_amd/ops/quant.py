"""Fake-quantization ops (HIP kernels on the GPU, torch on the CPU) with straight-through gradients.

Reference behaviour: paddle/fluid/operators/fake_quantize_op.{h,cc,cu.h} (fake_quantize_* /
fake_quantize_dequantize_* / fake_channel_wise_* / moving_average_abs_max_scale, round_type 1 =
TiesAwayFromZero by default), fake_dequantize_op (fake_dequantize_max_abs,
fake_channel_wise_dequantize_max_abs) and quantize_linear_op (quantize_linear / dequantize_linear).
The backward of every quant-dequant op is the straight-through estimator (StrightThroughEstimator
GradKernel: dX = dOut).

Kernels: csrc/kernels/quant.hip (abs-max and channel abs-max reductions, quant / quant-dequant
pass, moving-average scale update). Scales are fp32 device tensors; nothing here synchronises
with the host."""
from __future__ import annotations

from ctypes import c_float, c_int, c_long, c_void_p

import torch

from . import _lib

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def _L():
    L = _lib._load()
    if L is None:
        raise RuntimeError(f"libpha_kernels.so not loaded: {_lib._load_error}")
    if not getattr(L, "_quant_sig", False):
        P, I, LG = c_void_p, c_int, c_long
        L.pha_quant_absmax.argtypes = [I, P, LG, P, P]
        L.pha_quant_channel_absmax.argtypes = [I, P, LG, LG, LG, P, P]
        L.pha_quant_dequant.argtypes = [I, I, P, P, LG, LG, LG, P, I, I, I, P]
        L.pha_quant_moving_avg.argtypes = [P, P, P, P, c_float, P]
        for f in (L.pha_quant_absmax, L.pha_quant_channel_absmax, L.pha_quant_dequant, L.pha_quant_moving_avg):
            f.restype = c_int
        L._quant_sig = True
    return L


def _native(x):
    if not x.is_cuda:
        return False
    if x.dtype not in _DT:
        return False
    return _lib.require_native()


def _prep(x):
    x = x.contiguous()
    return x if x.data_ptr() % 16 == 0 else x.clone()


def _st(x):
    return c_void_p(torch.cuda.current_stream(x.device).cuda_stream)


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc})")


def bin_cnt(bits):
    return float((1 << (int(bits) - 1)) - 1)


def _axis_view(shape, axis):
    axis = int(axis) % len(shape)   # negative quant_axis counts from the last dimension
    outer = 1
    for s in shape[:axis]:
        outer *= int(s)
    inner = 1
    for s in shape[axis + 1:]:
        inner *= int(s)
    return outer, int(shape[axis]), inner


# ----------------------------------------------------------------------------------- scales
def abs_max(x):
    """max |x| as a fp32 [1] tensor"""
    x = x.detach()
    if _native(x):
        x = _prep(x)
        out = torch.empty(1, dtype=torch.float32, device=x.device)
        _chk(_L().pha_quant_absmax(_DT[x.dtype], c_void_p(x.data_ptr()), x.numel(), c_void_p(out.data_ptr()), _st(x)),
             "pha_quant_absmax")
        return out
    return x.abs().max().float().reshape(1) if x.numel() else torch.zeros(1, device=x.device)


def channel_abs_max(x, quant_axis=0):
    """max |x| over everything but ``quant_axis`` -> fp32 [C]"""
    x = x.detach()
    outer, C, inner = _axis_view(x.shape, quant_axis)
    if _native(x):
        x = _prep(x)
        out = torch.empty(C, dtype=torch.float32, device=x.device)
        _chk(_L().pha_quant_channel_absmax(_DT[x.dtype], c_void_p(x.data_ptr()), outer, C, inner,
                                           c_void_p(out.data_ptr()), _st(x)), "pha_quant_channel_absmax")
        return out
    return x.abs().float().reshape(outer, C, inner).amax(dim=(0, 2))


def moving_average_update(cur, state, accum, scale, rate):
    """in place: state = r*state + 1, accum = r*accum + cur, scale = accum / state (fp32 [1] each)"""
    if cur.is_cuda and _lib.require_native():
        _chk(_L().pha_quant_moving_avg(*(c_void_p(t.data_ptr()) for t in (cur, state, accum, scale)), float(rate),
                                       _st(cur)), "pha_quant_moving_avg")
        return
    with torch.no_grad():
        state.mul_(rate).add_(1.0)
        accum.mul_(rate).add_(cur.to(accum.dtype))
        scale.copy_(accum / state)


# ----------------------------------------------------------------------------------- quantize
def _qdq_torch(x, scale, bits, round_type, dequant, C, inner):
    xf = x.float()
    bn = bin_cnt(bits)
    if C > 1:
        shape = [1] * x.dim()
        s = scale.float().reshape(-1)
        xs = xf.reshape(-1, C, inner)
        s = s.reshape(1, C, 1)
    else:
        xs = xf
        s = scale.float().reshape(())
    inv = torch.where(s <= 1e-30, 1.0 / (s + 1e-6), 1.0 / s)
    if round_type == 0:
        q = torch.clamp(torch.round(bn * inv * xs), -bn - 1, bn)   # torch.round: ties to even
    else:
        v = torch.maximum(torch.minimum(xs, s), -s) * bn * inv
        q = torch.sign(v) * torch.floor(v.abs() + 0.5)                # ties away from zero
    out = q * s / bn if dequant else q
    return out.reshape(x.shape)


def quant_dequant(x, scale, bits=8, round_type=1, dequant=True, quant_axis=None, out_dtype=None):
    """fake quant(-dequant) of x with a per-tensor ([1]) or per-channel ([C] along quant_axis) scale"""
    x = x.detach()
    if quant_axis is None or scale.numel() == 1:
        C, inner = 1, 1
    else:
        _, C, inner = _axis_view(x.shape, quant_axis)
    od = out_dtype or x.dtype
    if _native(x) and od in (x.dtype, torch.float32):
        x = _prep(x)
        scale = scale.detach().float().contiguous()
        y = torch.empty(x.shape, dtype=od, device=x.device)
        _chk(_L().pha_quant_dequant(_DT[x.dtype], _DT[od], c_void_p(x.data_ptr()), c_void_p(y.data_ptr()), x.numel(),
                                    C, inner, c_void_p(scale.data_ptr()), int(bits), int(round_type), int(dequant),
                                    _st(x)), "pha_quant_dequant")
        return y
    return _qdq_torch(x, scale, bits, round_type, dequant, C, inner).to(od)


class _STE(torch.autograd.Function):
    """forward: the quant-dequant value; backward: dX = dOut (straight-through estimator)"""

    @staticmethod
    def forward(ctx, x, y):
        return y

    @staticmethod
    def backward(ctx, g):
        return g, None


def ste(x, y):
    """y (computed without autograd) with x's gradient passed straight through"""
    if torch.is_grad_enabled() and x.requires_grad:
        return _STE.apply(x, y)
    return y


# ------------------------------------------------------------- the reference op set (torch level)
def fake_quantize_dequantize_abs_max(x, bits=8, round_type=1):
    """-> (out, out_scale[1])"""
    s = abs_max(x)
    return ste(x, quant_dequant(x, s, bits, round_type)), s


def fake_quantize_abs_max(x, bits=8, round_type=1):
    """-> (integer levels in x's float dtype, scale[1])"""
    s = abs_max(x)
    return quant_dequant(x, s, bits, round_type, dequant=False), s


def fake_channel_wise_quantize_dequantize_abs_max(x, bits=8, quant_axis=0, round_type=1):
    s = channel_abs_max(x, quant_axis)
    return ste(x, quant_dequant(x, s, bits, round_type, quant_axis=quant_axis)), s


def fake_channel_wise_quantize_abs_max(x, bits=8, quant_axis=0, round_type=1):
    s = channel_abs_max(x, quant_axis)
    return quant_dequant(x, s, bits, round_type, dequant=False, quant_axis=quant_axis), s


def fake_quantize_dequantize_moving_average_abs_max(x, scale, state, accum, bits=8, moving_rate=0.9, is_test=False,
                                                    round_type=1):
    """training: the scale follows the moving average of max|x| (updated in place); test: the stored
    scale quantizes"""
    if not is_test:
        moving_average_update(abs_max(x), state, accum, scale, moving_rate)
    return ste(x, quant_dequant(x, scale, bits, round_type))


def fake_quantize_moving_average_abs_max(x, scale, state, accum, bits=8, moving_rate=0.9, is_test=False,
                                         round_type=1):
    if not is_test:
        moving_average_update(abs_max(x), state, accum, scale, moving_rate)
    return quant_dequant(x, scale, bits, round_type, dequant=False)


def moving_average_abs_max_scale(x, scale, state, accum, moving_rate=0.9, is_test=False):
    """records the moving-average output scale of x; x passes through"""
    if not is_test:
        moving_average_update(abs_max(x), state, accum, scale, moving_rate)
    return x


def fake_dequantize_max_abs(x, scale, max_range):
    """out = x * scale / max_range"""
    return x * (scale.reshape(()).to(x.dtype) / float(max_range))


def fake_channel_wise_dequantize_max_abs(x, scales, quant_bits=(8,), quant_axis=0):
    """out = x * scale[c] / (2^(bits-1) - 1) along quant_axis (one scale set)"""
    _, C, inner = _axis_view(x.shape, quant_axis)
    s = scales.float().reshape(1, C, 1) / bin_cnt(quant_bits[0])
    return (x.float().reshape(-1, C, inner) * s).reshape(x.shape).to(x.dtype)


class _ScaledSTE(torch.autograd.Function):
    """forward: y (computed without autograd); backward: dX = dY * factor (the quantize step's
    straight-through derivative bin / s)"""

    @staticmethod
    def forward(ctx, x, y, factor):
        ctx.save_for_backward(factor)
        return y

    @staticmethod
    def backward(ctx, g):
        f, = ctx.saved_tensors
        return g * f.to(g.dtype), None, None


def quantize_linear(x, scale, zero_point=None, bit_length=8, quant_axis=-1, round_type=0):
    """the 2.4 export op: q = clip(round(x / s * bin) + zp) (integer levels, x's float dtype)"""
    per_ch = scale.numel() > 1
    q = quant_dequant(x, scale, bit_length, round_type, dequant=False, quant_axis=quant_axis if per_ch else None)
    if torch.is_grad_enabled() and x.requires_grad and x.is_floating_point():
        s = scale.detach().float()
        if per_ch:
            s = s.reshape([-1 if i == quant_axis % x.dim() else 1 for i in range(x.dim())])
        q = _ScaledSTE.apply(x, q.to(x.dtype), bin_cnt(bit_length) / torch.where(s <= 1e-30, s + 1e-6, s))
    if zero_point is not None and bool((zero_point != 0).any()):
        q = q + zero_point.to(q.dtype).reshape([-1 if i == quant_axis % x.dim() else 1 for i in range(x.dim())]
                                                if per_ch else [])
    return q


def dequantize_linear(q, scale, zero_point=None, bit_length=8, quant_axis=-1):
    bn = bin_cnt(bit_length)
    per_ch = scale.numel() > 1
    if zero_point is not None and bool((zero_point != 0).any()):
        q = q - zero_point.to(q.dtype).reshape([-1 if i == quant_axis % q.dim() else 1 for i in range(q.dim())]
                                                if per_ch else [])
    if per_ch:
        shape = [-1 if i == quant_axis % q.dim() else 1 for i in range(q.dim())]
        return (q.float() * scale.float().reshape(shape) / bn).to(q.dtype if q.is_floating_point() else torch.float32)
    return (q.float() * scale.float().reshape(()) / bn).to(q.dtype if q.is_floating_point() else torch.float32)
