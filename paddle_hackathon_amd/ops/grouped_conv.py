"""Direct NHWC convolution on the gfx950 HIP kernels of csrc/kernels/grouped_conv.hip: grouped and
depthwise convolutions, dilated + strided ones, fp32 grouped ones — the layouts the implicit-GEMM
MFMA kernels (ops/conv_gemm.py) do not take. Reference: phi/kernels/gpu/conv_kernel.cu (grouped
path), phi/kernels/gpu/depthwise_conv.h and depthwise_conv_grad_kernel.cu.

Weights keep Paddle's [C_out, C_in / groups, KH, KW]; the forward re-lays them out once per call as
[KH][KW][C_in/groups][C_out] (8 output channels = one vector), the input gradient as
[KH][KW][C_out][C_in/groups]. Channel counts must be multiples of 8 (``supported``); dense
(groups == 1) and depthwise convolutions with other counts are zero-padded to them.
"""
from __future__ import annotations

from ctypes import c_int, c_long, c_void_p

import torch

from . import _lib

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def _L():
    L = _lib._load()
    if L is None:
        raise RuntimeError(f"libpha_kernels.so not loaded: {_lib._load_error}")
    if not getattr(L, "_gconv_sig", False):
        P = c_void_p
        L.pha_gconv_fwd.argtypes = [c_int, P, P, P, P, P, P]
        L.pha_gconv_fwd.restype = c_int
        L.pha_gconv_dgrad.argtypes = [c_int, P, P, P, P, P]
        L.pha_gconv_dgrad.restype = c_int
        L.pha_gconv_wgrad_ws.argtypes = [P, c_int]
        L.pha_gconv_wgrad_ws.restype = c_long
        L.pha_gconv_wgrad_items.argtypes = [P]
        L.pha_gconv_wgrad_items.restype = c_long
        L.pha_gconv_wgrad.argtypes = [c_int, P, P, P, P, P, c_int, P]
        L.pha_gconv_wgrad.restype = c_int
        L._gconv_sig = True
    return L


def _p(t):
    return c_void_p(0 if t is None else t.data_ptr())


def _stream(t):
    return c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"pha_gconv_{what} failed ({rc})")


def out_size(size, k, s, p, d):
    return (size + 2 * p - d * (k - 1) - 1) // s + 1


def supported(x, w, groups):
    """x NHWC, w [C_out, C_in/groups, KH, KW]"""
    return (x.is_cuda and x.dim() == 4 and w.dim() == 4 and x.dtype in _DT and w.dtype == x.dtype
            and x.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0 and x.shape[-1] == w.shape[1] * groups
            and w.shape[0] % groups == 0 and _lib.native_available())


def _dims(x, w, stride, pad, dil, groups):
    N, H, W, C = x.shape
    CO, _, KH, KW = w.shape
    OH, OW = out_size(H, KH, stride[0], pad[0], dil[0]), out_size(W, KW, stride[1], pad[1], dil[1])
    d = [N, H, W, C, OH, OW, CO, KH, KW, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], groups]
    return torch.tensor(d, dtype=torch.int32), (N, OH, OW, CO)


class GroupedConv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, stride, pad, dil, groups):
        x = x.contiguous()
        dims, oshape = _dims(x, w, stride, pad, dil, groups)
        if min(oshape) <= 0:
            raise ValueError(f"conv2d output shape {oshape} is empty")
        wr = w.permute(2, 3, 1, 0).contiguous()
        y = torch.empty(oshape, dtype=x.dtype, device=x.device)
        b = None if bias is None else bias.float().contiguous()
        _check(_L().pha_gconv_fwd(_DT[x.dtype], _p(dims), _p(x), _p(wr), _p(b), _p(y), _stream(x)), "fwd")
        ctx.save_for_backward(x, w)
        ctx.conf = (stride, pad, dil, groups, bias is not None)
        ctx.dims = dims
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, pad, dil, groups, has_b = ctx.conf
        dims = ctx.dims
        gy = gy.contiguous()
        L = _L()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            depthwise = w.shape[1] == 1 and w.shape[0] == groups
            w2 = w.permute(2, 3, 1, 0).contiguous() if depthwise else w.permute(2, 3, 0, 1).contiguous()
            dx = torch.empty_like(x)
            _check(L.pha_gconv_dgrad(_DT[x.dtype], _p(dims), _p(gy), _p(w2), _p(dx), _stream(x)), "dgrad")
        if ctx.needs_input_grad[1]:
            base = L.pha_gconv_wgrad_items(_p(dims))
            npix = gy.shape[0] * gy.shape[1] * gy.shape[2]
            chunks = max(1, min(-(-2048 // base), -(-npix // 256)))
            ws = torch.empty(L.pha_gconv_wgrad_ws(_p(dims), chunks), dtype=torch.float32, device=x.device)
            dw = torch.empty_like(w)
            _check(L.pha_gconv_wgrad(_DT[x.dtype], _p(dims), _p(x), _p(gy), _p(dw), _p(ws), chunks, _stream(x)),
                   "wgrad")
        if has_b and ctx.needs_input_grad[2]:
            g2 = gy.reshape(-1, gy.shape[-1])
            if gy.dtype in (torch.bfloat16, torch.float16) and g2.shape[1] % 8 == 0:
                from . import hip
                db = hip.col_sum(g2)
            else:
                db = g2.float().sum(0).to(gy.dtype)
        return dx, dw, db, None, None, None, None


class GroupedConvTranspose2dNHWC(torch.autograd.Function):
    """y = conv_transpose(x, w): the input gradient of the convolution F whose weight is w
    ([C_in, C_out / groups, KH, KW] read as F's [C_out', C_in' / groups, KH, KW]) applied to x;
    dx = F(dy), dw = F's filter gradient with (input dy, output gradient x)."""

    @staticmethod
    def forward(ctx, x, w, bias, stride, pad, dil, groups, out_hw):
        x = x.contiguous()
        N, H, W, Cin = x.shape
        Cout = w.shape[1] * groups
        OH, OW = out_hw
        d = [N, OH, OW, Cout, H, W, Cin, w.shape[2], w.shape[3], stride[0], stride[1], pad[0], pad[1], dil[0], dil[1],
             groups]
        dims = torch.tensor(d, dtype=torch.int32)
        depthwise = w.shape[1] == 1 and w.shape[0] == groups
        w2 = w.permute(2, 3, 1, 0).contiguous() if depthwise else w.permute(2, 3, 0, 1).contiguous()
        y = torch.empty(N, OH, OW, Cout, dtype=x.dtype, device=x.device)
        _check(_L().pha_gconv_dgrad(_DT[x.dtype], _p(dims), _p(x), _p(w2), _p(y), _stream(x)), "dgrad")
        if bias is not None:
            y += bias.to(y.dtype)
        ctx.save_for_backward(x, w)
        ctx.dims, ctx.has_b = dims, bias is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        dims = ctx.dims
        gy = gy.contiguous()
        L = _L()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wr = w.permute(2, 3, 1, 0).contiguous()
            dx = torch.empty_like(x)
            _check(L.pha_gconv_fwd(_DT[x.dtype], _p(dims), _p(gy), _p(wr), None, _p(dx), _stream(x)), "fwd")
        if ctx.needs_input_grad[1]:
            base = L.pha_gconv_wgrad_items(_p(dims))
            npix = x.shape[0] * x.shape[1] * x.shape[2]
            chunks = max(1, min(-(-2048 // base), -(-npix // 256)))
            ws = torch.empty(L.pha_gconv_wgrad_ws(_p(dims), chunks), dtype=torch.float32, device=x.device)
            dw = torch.empty_like(w)
            _check(L.pha_gconv_wgrad(_DT[x.dtype], _p(dims), _p(gy), _p(x), _p(dw), _p(ws), chunks, _stream(x)),
                   "wgrad")
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = gy.reshape(-1, gy.shape[-1]).float().sum(0).to(gy.dtype)
        return dx, dw, db, None, None, None, None, None


def conv_transpose2d_nhwc(x, w, bias, stride, pad, dil, groups, out_hw):
    """NHWC transposed convolution on the direct kernels (channel counts multiples of 8)"""
    return GroupedConvTranspose2dNHWC.apply(x, w, bias, tuple(stride), tuple(pad), tuple(dil), groups, tuple(out_hw))


def transpose_ok(x, w, groups):
    return (x.is_cuda and x.dim() == 4 and w.dim() == 4 and x.dtype in _DT and w.dtype == x.dtype
            and x.shape[-1] == w.shape[0] and x.shape[-1] % 8 == 0 and (w.shape[1] * groups) % 8 == 0
            and x.shape[-1] % groups == 0 and _lib.native_available())


def conv2d_nhwc(x, w, bias, stride, pad, dil, groups):
    """NHWC direct convolution; a dense one whose channel counts are not multiples of 8 is
    zero-padded (input channels of x and w, output channels of w, sliced off the result)"""
    C, CO = x.shape[-1], w.shape[0]
    if groups == C and w.shape[1] == 1 and C % 8:
        # depthwise (multiplier m = CO / C): the padded channels are extra groups of zeros
        m = CO // C
        cp = -(-C // 8) * 8
        x = torch.nn.functional.pad(x, [0, cp - C])
        w = torch.nn.functional.pad(w, [0, 0, 0, 0, 0, 0, 0, (cp - C) * m])
        if bias is not None:
            bias = torch.nn.functional.pad(bias, [0, (cp - C) * m])
        return GroupedConv2dNHWC.apply(x, w, bias, tuple(stride), tuple(pad), tuple(dil), cp)[..., :CO]
    if groups == 1 and (C % 8 or CO % 8):
        cp, op = -(-C // 8) * 8, -(-CO // 8) * 8
        x = torch.nn.functional.pad(x, [0, cp - C])
        w = torch.nn.functional.pad(w, [0, 0, 0, 0, 0, cp - C, 0, op - CO])
        if bias is not None:
            bias = torch.nn.functional.pad(bias, [0, op - CO])
        return GroupedConv2dNHWC.apply(x, w, bias, tuple(stride), tuple(pad), tuple(dil), 1)[..., :CO]
    return GroupedConv2dNHWC.apply(x, w, bias, tuple(stride), tuple(pad), tuple(dil), groups)


def ok(x, w, groups):
    """the direct kernel takes (x NHWC, w): grouped convolutions of any dtype with channel counts
    that are multiples of 8, dense bf16 / fp16 ones of any channel count (zero-padded). Dense fp32
    convolutions are left to the caller: per output channel they are C_in * KH * KW FMAs on the
    vector ALUs, where MIOpen's fp32 kernels are the better tool."""
    if not (x.is_cuda and x.dim() == 4 and w.dim() == 4 and x.dtype in _DT and w.dtype == x.dtype
            and _lib.native_available()):
        return False
    if groups == 1:
        return x.dtype != torch.float32
    if groups == x.shape[-1] and w.shape[1] == 1 and w.shape[0] % groups == 0:
        return True    # depthwise: padded to 8 channels when needed
    return supported(x, w, groups)
