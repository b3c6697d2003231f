"""Convolutions (reference: python/paddle/nn/functional/conv.py, phi/kernels/gpu/conv_*).

Paddle layouts: weight [C_out, C_in/groups, *k] (transpose conv: [C_in, C_out/groups, *k]);
``data_format`` NCHW or NHWC. 2-D convolutions run on the own kernels in NHWC memory for both
formats (``_own_conv2d``), fp32 ones included (a three-term bf16 split on the same MFMA kernels,
ops/conv_gemm.py split3); 1-D convolutions run as height-1 2-D ones, 3-D ones as one 2-D
convolution per depth tap (``_conv3d_as_2d``). What they do not take (some transposed / grouped /
"SAME"-padded forms) goes to MIOpen and is counted by ops/fallback.py.
"""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _wrap
from ...framework.dispatch import register_ops

_w = _wrap

__all__ = ["conv1d", "conv2d", "conv3d", "conv1d_transpose", "conv2d_transpose", "conv3d_transpose"]


def _tup(v, n):
    if isinstance(v, (list, tuple)):
        v = [int(a) for a in v]
        if len(v) == 1:
            return v * n
        return v
    return [int(v)] * n


def _padding(padding, n, k, stride, dilation, x_spatial):
    """Paddle padding forms -> (torch_padding, pre_pad list or None)."""
    if isinstance(padding, str):
        p = padding.upper()
        if p == "VALID":
            return [0] * n, None
        if p == "SAME":
            pads = []
            for i in range(n):
                out = (x_spatial[i] + stride[i] - 1) // stride[i]
                tot = max((out - 1) * stride[i] + (k[i] - 1) * dilation[i] + 1 - x_spatial[i], 0)
                pads.append((tot // 2, tot - tot // 2))
            if all(a == b for a, b in pads):
                return [a for a, _ in pads], None
            return [0] * n, pads
        raise ValueError(padding)
    if isinstance(padding, (list, tuple)):
        padding = list(padding)
        if len(padding) == n and all(isinstance(p, int) for p in padding):
            return padding, None
        if len(padding) == 2 * n and all(isinstance(p, int) for p in padding):
            pads = [(padding[2 * i], padding[2 * i + 1]) for i in range(n)]
            if all(a == b for a, b in pads):
                return [a for a, _ in pads], None
            return [0] * n, pads
        if len(padding) == n + 2:  # [[0,0],[0,0],[a,b],...] forms
            sp = [p for p in padding if list(p) != [0, 0]] if len(padding) else []
            flat = [tuple(p) for p in padding]
            spatial = flat[2:] if flat[1] == (0, 0) else flat[1:-1]
            return _padding([v for pr in spatial for v in pr], n, k, stride, dilation, x_spatial)
    return [int(padding)] * n, None


def _to_ncx(t, data_format):
    if data_format[-1] == "C" and len(data_format) > 2:
        return t.movedim(-1, 1), True
    return t, False


def _s2d_ok(x, w, stride, dilation):
    import os
    s = stride[0]
    C = x.shape[-1]
    return (os.environ.get("PHA_CONV_S2D", "1") != "0" and C % 8 != 0 and s > 1 and stride[1] == s
            and tuple(dilation) == (1, 1) and w.shape[2] > s and w.shape[3] > s and s * s * C <= 32
            and x.dtype in (torch.bfloat16, torch.float16))


def _space_to_depth(x, w, stride, pad):
    """a stride-s convolution of a narrow input (the RGB stem: C = 3, 7x7, stride 2) rewritten as a
    stride-1 convolution of the input's s x s space-to-depth image — channel (a, b, c) of pixel
    (hq, wq) holds padded-input pixel (s*hq + a, s*wq + b), channel c — with the filter's taps
    regrouped the same way (ceil(k/s)^2 taps of s*s*c' channels, zero taps past k). The stem's
    implicit GEMM then reduces over K = 4*4*16 = 256 instead of 7*7*8 = 392 (the input padded to 8
    channels) and reads 32-B tap rows instead of 16-B ones. Returns (image, filter) for a stride-1,
    unpadded convolution with the same output."""
    N, H, W, C = x.shape
    Co, _, KH, KW = w.shape
    s = stride[0]
    ph, pw = pad
    kh, kw = -(-KH // s), -(-KW // s)
    OH, OW = (H + 2 * ph - KH) // s + 1, (W + 2 * pw - KW) // s + 1
    Hq, Wq = OH + kh - 1, OW + kw - 1
    c4 = C
    while (s * s * c4) % 8:
        c4 += 1
    z = x.new_zeros(N, Hq, Wq, s, s, c4)
    for a in range(s):
        hq0 = max(0, -(-(ph - a) // s))
        r0 = s * hq0 + a - ph
        nh = min(Hq - hq0, len(range(r0, H, s)))
        for b in range(s):
            wq0 = max(0, -(-(pw - b) // s))
            q0 = s * wq0 + b - pw
            nw = min(Wq - wq0, len(range(q0, W, s)))
            if nh > 0 and nw > 0:
                z[:, hq0:hq0 + nh, wq0:wq0 + nw, a, b, :C] = \
                    x[:, r0:r0 + s * (nh - 1) + 1:s, q0:q0 + s * (nw - 1) + 1:s, :]
    wp = TF.pad(w, [0, s * kw - KW, 0, s * kh - KH, 0, c4 - C])          # [Co, c4, s*kh, s*kw]
    wz = wp.view(Co, c4, kh, s, kw, s).permute(0, 3, 5, 1, 2, 4).reshape(Co, s * s * c4, kh, kw)
    return z.view(N, Hq, Wq, s * s * c4), wz


def _hip_conv2d(x, w, bias, stride, pad, dilation, groups):
    """NHWC conv on the gfx950 implicit-GEMM MFMA kernels (ops/conv_gemm.py: forward, dgrad and
    wgrad on the 256-tile glds kernels of gemm256.hip; PHA_CONV_KERNEL=v1 selects the older
    gemm_conv.hip path). Narrow strided inputs (the RGB stem) run as the stride-1 convolution of
    their space-to-depth image (``_space_to_depth``, PHA_CONV_S2D=0: off); other inputs whose
    channel count is not a multiple of 8 are zero-padded to 8 channels."""
    import os
    from ...ops import conv_gemm
    if _s2d_ok(x, w, stride, dilation) and os.environ.get("PHA_CONV_KERNEL", "256") != "v1":
        z, wz = _space_to_depth(x, w, list(stride), list(pad))
        return conv_gemm.conv2d_nhwc256(z, wz, bias, (1, 1), (0, 0), (1, 1))
    if x.shape[-1] % 8 != 0:
        c = x.shape[-1]
        cp = (c + 7) // 8 * 8
        x = TF.pad(x, [0, cp - c])
        w = TF.pad(w, [0, 0, 0, 0, 0, cp - c])
    if x.dtype == torch.float32:   # fp32: three-term bf16 split on the same MFMA kernels
        return conv_gemm.conv2d_nhwc256_f32(x, w, bias, stride, pad, dilation)
    if os.environ.get("PHA_CONV_KERNEL", "256") == "v1":
        return conv_gemm.conv2d_nhwc(x, w, bias, stride, pad, dilation)
    return conv_gemm.conv2d_nhwc256(x, w, bias, stride, pad, dilation)


def _hip_conv_ok(t_nhwc, w, groups):
    import os
    # NHWC bf16/fp16 convs run on the MFMA implicit-GEMM kernels (ResNet-50 at batch 256: 7.46k img/s
    # vs 7.35k with MIOpen, profiles/README.md); PHA_CONV_IMPL=library selects MIOpen instead.
    if os.environ.get("PHA_CONV_IMPL", "hip") != "hip":
        return False
    from ...ops import conv_gemm, _lib
    # fp32 dense convs: the same kernels over a three-term bf16 split (conv_gemm.split3); PHA_CONV_F32=library
    # keeps them on MIOpen
    f32 = t_nhwc.dtype == torch.float32 and os.environ.get("PHA_CONV_F32", "hip") == "hip"
    return (t_nhwc.is_cuda and t_nhwc.dim() == 4 and (t_nhwc.dtype in (torch.bfloat16, torch.float16) or f32)
            and w.dtype == t_nhwc.dtype and groups == 1 and w.shape[0] % 8 == 0 and _lib.require_native())


def _own_conv2d(t, w, bias, stride, padding, dilation, groups, data_format):
    """2-D convolution on the own HIP kernels, or None when they do not take it.

    Physical layout is NHWC either way: an NCHW input is viewed through ``permute(0, 2, 3, 1)``
    (free when it is already channels-last in memory, one transpose otherwise — typically only the
    network's input) and the NHWC result is returned as an NCHW view (channels-last memory), so a
    whole NCHW network stays channels-last after its first layer: BN, pooling and the following
    convolutions see NHWC memory again (``nhwc_view``).
    Dense bf16 / fp16 convolutions run on the implicit-GEMM MFMA kernels (ops/conv_gemm.py);
    grouped / depthwise, dilated + strided and fp32 grouped ones on the direct kernels
    (ops/grouped_conv.py)."""
    import os
    if os.environ.get("PHA_CONV_IMPL", "hip") != "hip" or not t.is_cuda or t.dim() != 4:
        return None
    nchw = data_format == "NCHW"
    x = t.permute(0, 2, 3, 1) if nchw else t
    st, dl = _tup(stride, 2), _tup(dilation, 2)
    pad, pre = _padding(padding, 2, list(w.shape[2:]), st, dl, list(x.shape[1:3]))
    from ...ops import grouped_conv as _gc
    CO = w.shape[0]
    wp, bp = w, bias
    if groups == 1 and CO % 8:   # output channels padded to 8 with zero filters, sliced off below
        wp = TF.pad(w, [0, 0, 0, 0, 0, 0, 0, -CO % 8])
        bp = None if bias is None else TF.pad(bias, [0, -CO % 8])
    dense = _hip_conv_ok(x, wp, groups) and (st == [1, 1] or dl == [1, 1])
    from ...ops import conv_gemm as _cgm
    gmfma = (not dense and groups > 1 and w.shape[1] != 1
             and (st == [1, 1] or dl == [1, 1]) and _cgm.grouped_ok(x, w, groups))
    if not dense and not gmfma and not _gc.ok(x, w, groups):
        return None
    x = x.contiguous()
    if pre is not None:   # asymmetric ("SAME") padding: explicit zero rows / columns
        x = TF.pad(x, [0, 0, pre[1][0], pre[1][1], pre[0][0], pre[0][1]])
        pad = [0, 0]
    if dense:
        out = _hip_conv2d(x, wp, bp, st, pad, dl, groups)
        if out.shape[-1] != CO:
            out = out[..., :CO]
    elif gmfma:   # grouped (ResNeXt-style) convs: one grouped implicit GEMM per pass on the matrix cores
        out = _cgm.conv2d_nhwc256_grouped(x, w, bias, st, pad, dl, groups)
    else:
        out = _gc.conv2d_nhwc(x, w, bias, st, pad, dl, groups)
    return out.permute(0, 3, 1, 2) if nchw else out


def nhwc_view(t):
    """the NHWC tensor whose permute is the 4-D NCHW tensor ``t`` when ``t`` is channels-last in
    memory (what the own convolutions return), else None"""
    if t.dim() != 4:
        return None
    v = t.permute(0, 2, 3, 1)
    return v if v.is_contiguous() else None


def _conv1d_as_2d(t, w, bias, stride, padding, dilation, groups, data_format):
    """a 1-D convolution as the 2-D one over a height-1 image (the own kernels), or None"""
    if data_format not in ("NCL", "NLC") or t.dim() != 3:
        return None
    if isinstance(padding, str):
        pad2 = padding
    else:
        p = padding if isinstance(padding, (list, tuple)) else [padding]
        p = [int(v) for v in p]
        if len(p) == 1:
            pad2 = [0, p[0]]
        elif len(p) == 2:
            pad2 = [0, 0, p[0], p[1]]
        else:
            return None
    nchw = data_format == "NCL"
    x4 = t.unsqueeze(2) if nchw else t.unsqueeze(1)
    out = _own_conv2d(x4, w.unsqueeze(2), bias, [1, _tup(stride, 1)[0]], pad2, [1, _tup(dilation, 1)[0]], groups,
                      "NCHW" if nchw else "NHWC")
    if out is None:
        return None
    return out.squeeze(2) if nchw else out.squeeze(1)


def _conv3d_as_2d(t, w, bias, stride, padding, dilation, groups, data_format):
    """3-D convolution on the own 2-D kernels: out[:, od] = sum_kd conv2d(x[:, od*sd - pd + kd*dd],
    w[:, :, kd]) — one height x width convolution per depth tap over all (batch, output-depth)
    planes at once, summed in fp32 (autograd runs through the 2-D convolutions). None when the
    2-D kernels do not take the planes."""
    if data_format not in ("NCDHW", "NDHWC") or t.dim() != 5 or isinstance(padding, str):
        return None
    st, dl = _tup(stride, 3), _tup(dilation, 3)
    k = list(w.shape[2:])
    pad, pre = _padding(padding, 3, k, st, dl, [0, 0, 0])
    if pre is not None:
        return None
    x = t.permute(0, 2, 3, 4, 1) if data_format == "NCDHW" else t     # N, D, H, W, C
    N, D, H, W, C = x.shape
    KD = k[0]
    OD = (D + 2 * pad[0] - dl[0] * (KD - 1) - 1) // st[0] + 1
    if OD <= 0:
        return None
    xp = TF.pad(x, [0, 0, 0, 0, 0, 0, pad[0], pad[0]]) if pad[0] else x
    acc = None
    for kd in range(KD):
        d0 = kd * dl[0]
        planes = xp[:, d0:d0 + (OD - 1) * st[0] + 1:st[0]].reshape(N * OD, H, W, C)
        o = _own_conv2d(planes, w[:, :, kd], None, st[1:], pad[1:], dl[1:], groups, "NHWC")
        if o is None:
            return None
        o = o.float() if o.dtype in (torch.bfloat16, torch.float16) else o   # fp32 sum of the taps
        acc = o if acc is None else acc + o
    out = acc.to(t.dtype)
    out = out.reshape(N, OD, out.shape[1], out.shape[2], out.shape[3])
    if bias is not None:
        out = out + bias
    return out.permute(0, 4, 1, 2, 3) if data_format == "NCDHW" else out


def _convnd(n, x, weight, bias, stride, padding, dilation, groups, data_format):
    t = x._t
    w = weight._t
    if n == 2 and data_format in ("NCHW", "NHWC"):
        out = _own_conv2d(t, w, None if bias is None else bias._t, stride, padding, dilation, groups, data_format)
        if out is not None:
            return _w(out)
    if n == 1 and t.is_cuda:
        out = _conv1d_as_2d(t, w, None if bias is None else bias._t, stride, padding, dilation, groups, data_format)
        if out is not None:
            return _w(out)
    if n == 3 and t.is_cuda:
        out = _conv3d_as_2d(t, w, None if bias is None else bias._t, stride, padding, dilation, groups, data_format)
        if out is not None:
            return _w(out)
    if t.is_cuda:
        from ...ops import fallback
        fallback.note(f"conv{n}d", f"{data_format} {t.dtype} groups={groups} -> MIOpen")
    t, cl = _to_ncx(t, data_format)
    stride = _tup(stride, n)
    dilation = _tup(dilation, n)
    k = list(w.shape[2:])
    pad, pre = _padding(padding, n, k, stride, dilation, list(t.shape[2:]))
    if pre is not None:
        fl = []
        for a, b in reversed(pre):
            fl += [a, b]
        t = TF.pad(t, fl)
    if cl and n == 2:
        t = t.contiguous(memory_format=torch.channels_last) if not t.is_contiguous(memory_format=torch.channels_last) else t
    f = {1: TF.conv1d, 2: TF.conv2d, 3: TF.conv3d}[n]
    out = f(t, w, None if bias is None else bias._t, stride, pad, dilation, groups)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


def conv1d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCL", name=None):
    return _convnd(1, x, weight, bias, stride, padding, dilation, groups, data_format)


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCHW", name=None):
    return _convnd(2, x, weight, bias, stride, padding, dilation, groups, data_format)


def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCDHW", name=None):
    return _convnd(3, x, weight, bias, stride, padding, dilation, groups, data_format)


def _own_conv2d_t(t, w, bias, stride, padding, output_padding, groups, dilation, output_size, data_format):
    """2-D transposed convolution on the own kernels (NHWC memory, as ``_own_conv2d``), or None.
    Dense bf16 / fp16: the input gradient of the convolution with the same weight on the 256-tile
    implicit-GEMM kernels; grouped / depthwise / dilated + strided: the direct kernels."""
    import os
    if os.environ.get("PHA_CONV_IMPL", "hip") != "hip" or not t.is_cuda or t.dim() != 4:
        return None
    nchw = data_format == "NCHW"
    x = t.permute(0, 2, 3, 1) if nchw else t
    st, dl = _tup(stride, 2), _tup(dilation, 2)
    k = list(w.shape[2:])
    if isinstance(padding, str):
        pad = [0, 0] if padding.upper() == "VALID" else [((k[i] - 1) * dl[i]) // 2 for i in range(2)]
    else:
        pad, pre = _padding(padding, 2, k, st, dl, list(x.shape[1:3]))
        if pre is not None:
            return None
    opad = _tup(output_padding, 2)
    H, W = x.shape[1], x.shape[2]
    base = [(H - 1) * st[0] - 2 * pad[0] + dl[0] * (k[0] - 1) + 1, (W - 1) * st[1] - 2 * pad[1] + dl[1] * (k[1] - 1) + 1]
    if output_size is not None:
        osz = _tup(output_size if not isinstance(output_size, Tensor) else output_size._t.tolist(), 2)
    else:
        osz = [base[0] + opad[0], base[1] + opad[1]]
    if any(o < b or o >= b + s for o, b, s in zip(osz, base, st)):
        return None
    from ...ops import grouped_conv as _gc, conv_gemm as _cg
    Cout = w.shape[1] * groups
    dense = (groups == 1 and x.dtype in (torch.bfloat16, torch.float16) and w.dtype == x.dtype
             and x.shape[-1] % 8 == 0 and Cout % 8 == 0 and (st == [1, 1] or dl == [1, 1])
             and _hip_conv_ok(x, w, 1))
    if dense:
        out = _cg.conv_transpose2d_nhwc256(x.contiguous(), w, bias, st, pad, dl, osz)
    elif _gc.transpose_ok(x, w, groups) and (groups > 1 or x.dtype != torch.float32):
        out = _gc.conv_transpose2d_nhwc(x, w, bias, st, pad, dl, groups, osz)
    else:
        return None
    return out.permute(0, 3, 1, 2) if nchw else out


def _convnd_t(n, x, weight, bias, stride, padding, output_padding, groups, dilation, output_size, data_format):
    t = x._t
    w = weight._t
    if n == 2 and data_format in ("NCHW", "NHWC"):
        out = _own_conv2d_t(t, w, None if bias is None else bias._t, stride, padding, output_padding, groups,
                            dilation, output_size, data_format)
        if out is not None:
            return _w(out)
    if t.is_cuda:
        from ...ops import fallback
        fallback.note(f"conv{n}d", f"{data_format} {t.dtype} groups={groups} -> MIOpen")
    t, cl = _to_ncx(t, data_format)
    stride = _tup(stride, n)
    dilation = _tup(dilation, n)
    k = list(w.shape[2:])
    if isinstance(padding, str):
        pad = [0] * n if padding.upper() == "VALID" else [((k[i] - 1) * dilation[i]) // 2 for i in range(n)]
    else:
        pad, pre = _padding(padding, n, k, stride, dilation, list(t.shape[2:]))
    opad = _tup(output_padding, n)
    if output_size is not None:
        osz = _tup(output_size if not isinstance(output_size, Tensor) else output_size._t.tolist(), n)
        for i in range(n):
            base = (t.shape[2 + i] - 1) * stride[i] - 2 * pad[i] + dilation[i] * (k[i] - 1) + 1
            opad[i] = osz[i] - base
    f = {1: TF.conv_transpose1d, 2: TF.conv_transpose2d, 3: TF.conv_transpose3d}[n]
    out = f(t, w, None if bias is None else bias._t, stride, pad, opad, groups, dilation)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


def conv1d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     output_size=None, data_format="NCL", name=None):
    return _convnd_t(1, x, weight, bias, stride, padding, output_padding, groups, dilation, output_size, data_format)


def conv2d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, dilation=1, groups=1,
                     output_size=None, data_format="NCHW", name=None):
    return _convnd_t(2, x, weight, bias, stride, padding, output_padding, groups, dilation, output_size, data_format)


def conv3d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     output_size=None, data_format="NCDHW", name=None):
    return _convnd_t(3, x, weight, bias, stride, padding, output_padding, groups, dilation, output_size, data_format)


register_ops(globals(), __all__)
