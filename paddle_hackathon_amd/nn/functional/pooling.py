"""Pooling (reference: python/paddle/nn/functional/pooling.py)."""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _wrap
from ...framework.dispatch import register_ops

_w = _wrap

__all__ = ["avg_pool1d", "avg_pool2d", "avg_pool3d", "max_pool1d", "max_pool2d", "max_pool3d",
           "adaptive_avg_pool1d", "adaptive_avg_pool2d", "adaptive_avg_pool3d", "adaptive_max_pool1d",
           "adaptive_max_pool2d", "adaptive_max_pool3d", "max_unpool1d", "max_unpool2d", "max_unpool3d",
           "lp_pool1d", "lp_pool2d"]


def _cl(t, data_format):
    if data_format in ("NHWC", "NLC", "NDHWC"):
        return t.movedim(-1, 1), True
    return t, False


def _pad_arg(padding, n, t, k, s, ceil_mode):
    if isinstance(padding, str):
        if padding.upper() == "VALID":
            return 0, None
        # SAME
        pads = []
        for i in range(n):
            size = t.shape[2 + i]
            out = (size + s[i] - 1) // s[i]
            tot = max((out - 1) * s[i] + k[i] - size, 0)
            pads.append((tot // 2, tot - tot // 2))
        if all(a == b for a, b in pads):
            return [a for a, _ in pads], None
        return 0, pads
    if isinstance(padding, (list, tuple)) and len(padding) == 2 * n:
        pads = [(padding[2 * i], padding[2 * i + 1]) for i in range(n)]
        if all(a == b for a, b in pads):
            return [a for a, _ in pads], None
        return 0, pads
    return padding, None


def _tup(v, n):
    if v is None:
        return None
    if isinstance(v, (list, tuple)):
        return [int(a) for a in v] if len(v) == n else [int(v[0])] * n
    return [int(v)] * n


def _pool(n, kind, x, kernel_size, stride, padding, ceil_mode, exclusive, divisor, data_format, return_mask=False):
    t, cl = _cl(x._t, data_format)
    k = _tup(kernel_size, n)
    s = _tup(stride, n) if stride is not None else k
    pad, pre = _pad_arg(padding, n, t, k, s, ceil_mode)
    if n == 2 and kind == "max" and pre is None and not ceil_mode and not return_mask:
        from ...ops import hip as _hip, fused as _fused
        from .conv import nhwc_view
        xt = x._t if cl else nhwc_view(x._t)   # NCHW in channels-last memory: its NHWC view
        p2 = list(_tup(pad, 2)) if not isinstance(pad, (list, tuple)) else list(pad)
        if xt is not None and len(p2) == 2 and _fused._use_hip(xt) and _hip.maxpool_nhwc_ok(xt, k, s, p2):
            # NHWC max pool on the HIP kernels (byte window index, gather backward)
            y = _hip.MaxPool2dNHWC.apply(xt, tuple(k), tuple(s), tuple(p2))
            return _w(y if cl else y.permute(0, 3, 1, 2))
    if pre is not None:
        fl = []
        for a, b in reversed(pre):
            fl += [a, b]
        t = TF.pad(t, fl, value=float("-inf") if kind == "max" else 0.0)
    if kind == "max":
        f = {1: TF.max_pool1d, 2: TF.max_pool2d, 3: TF.max_pool3d}[n]
        r = f(t, k, s, pad, 1, ceil_mode, return_mask)
        if return_mask:
            out, mask = r
            if cl:
                out, mask = out.movedim(1, -1), mask.movedim(1, -1)
            return _w(out), _w(mask)
        out = r
    else:
        # inclusive (exclusive=False) averages divide by the full kernel volume, also for ceil-mode
        # windows overhanging the padding (reference pool kernels / avg_pool2D_forward_naive);
        # torch's count_include_pad divides by the window clipped to the padded input
        if divisor is None and not exclusive:
            divisor = 1
            for v in k:
                divisor *= v
        if n == 1:
            p1 = pad if isinstance(pad, int) else (pad[0] if isinstance(pad, (list, tuple)) else 0)
            out = TF.avg_pool2d(t.unsqueeze(2), (1, k[0]), (1, s[0]), (0, p1), ceil_mode, not exclusive,
                                divisor).squeeze(2)
        else:
            f = TF.avg_pool2d if n == 2 else TF.avg_pool3d
            out = f(t, k, s, pad, ceil_mode, not exclusive, divisor)
    if ceil_mode and pre is None:
        out = _ceil_tail(out, t, k, s, pad, n, kind, exclusive)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


def _ceil_tail(out, t, k, s, pad, n, kind, exclusive):
    """ceil_mode output size as the reference computes it, (in - k + 2p + s - 1) / s + 1, which
    keeps a last window that starts inside the padding (torch drops it): pad the output with what
    the reference kernel yields for an empty window (0 inclusive avg, 0/0 exclusive avg, the
    max-pool initial value)"""
    pads = pad if isinstance(pad, (list, tuple)) else [pad] * n
    fl = []
    for i in reversed(range(n)):
        want = (t.shape[2 + i] - k[i] + 2 * int(pads[i]) + s[i] - 1) // s[i] + 1
        fl += [0, max(0, want - out.shape[2 + i])]
    if not any(fl):
        return out
    val = torch.finfo(out.dtype).min if kind == "max" else (float("nan") if exclusive else 0.0)
    return TF.pad(out, fl, value=val)


def avg_pool1d(x, kernel_size, stride=None, padding=0, exclusive=True, ceil_mode=False, name=None):
    return _pool(1, "avg", x, kernel_size, stride, padding, ceil_mode, exclusive, None, "NCL")


def avg_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
               data_format="NCHW", name=None):
    return _pool(2, "avg", x, kernel_size, stride, padding, ceil_mode, exclusive, divisor_override, data_format)


def avg_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
               data_format="NCDHW", name=None):
    return _pool(3, "avg", x, kernel_size, stride, padding, ceil_mode, exclusive, divisor_override, data_format)


def max_pool1d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, name=None):
    return _pool(1, "max", x, kernel_size, stride, padding, ceil_mode, True, None, "NCL", return_mask)


def max_pool2d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NCHW", name=None):
    return _pool(2, "max", x, kernel_size, stride, padding, ceil_mode, True, None, data_format, return_mask)


def max_pool3d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NCDHW", name=None):
    return _pool(3, "max", x, kernel_size, stride, padding, ceil_mode, True, None, data_format, return_mask)


def _adaptive(n, kind, x, output_size, data_format="NCHW", return_mask=False):
    t, cl = _cl(x._t, data_format)
    if isinstance(output_size, (list, tuple)):
        output_size = [t.shape[2 + i] if o is None else int(o) for i, o in enumerate(output_size)]
    if kind == "avg":
        f = {1: TF.adaptive_avg_pool1d, 2: TF.adaptive_avg_pool2d, 3: TF.adaptive_avg_pool3d}[n]
        out = f(t, output_size)
    else:
        f = {1: TF.adaptive_max_pool1d, 2: TF.adaptive_max_pool2d, 3: TF.adaptive_max_pool3d}[n]
        r = f(t, output_size, return_mask)
        if return_mask:
            return _w(r[0]), _w(r[1])
        out = r
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


def adaptive_avg_pool1d(x, output_size, name=None):
    return _adaptive(1, "avg", x, output_size, "NCL")


def adaptive_avg_pool2d(x, output_size, data_format="NCHW", name=None):
    return _adaptive(2, "avg", x, output_size, data_format)


def adaptive_avg_pool3d(x, output_size, data_format="NCDHW", name=None):
    return _adaptive(3, "avg", x, output_size, data_format)


def adaptive_max_pool1d(x, output_size, return_mask=False, name=None):
    return _adaptive(1, "max", x, output_size, "NCL", return_mask)


def adaptive_max_pool2d(x, output_size, return_mask=False, name=None):
    return _adaptive(2, "max", x, output_size, "NCHW", return_mask)


def adaptive_max_pool3d(x, output_size, return_mask=False, name=None):
    return _adaptive(3, "max", x, output_size, "NCDHW", return_mask)


def _unpool(n, x, indices, kernel_size, stride, padding, data_format, output_size):
    f = {1: TF.max_unpool1d, 2: TF.max_unpool2d, 3: TF.max_unpool3d}[n]
    osz = None if output_size is None else list(output_size)[-n:]
    return _w(f(x._t, indices._t, kernel_size, stride, padding, osz))


def max_unpool1d(x, indices, kernel_size, stride=None, padding=0, data_format="NCL", output_size=None, name=None):
    return _unpool(1, x, indices, kernel_size, stride, padding, data_format, output_size)


def max_unpool2d(x, indices, kernel_size, stride=None, padding=0, data_format="NCHW", output_size=None, name=None):
    return _unpool(2, x, indices, kernel_size, stride, padding, data_format, output_size)


def max_unpool3d(x, indices, kernel_size, stride=None, padding=0, data_format="NCDHW", output_size=None, name=None):
    return _unpool(3, x, indices, kernel_size, stride, padding, data_format, output_size)


def lp_pool1d(x, norm_type, kernel_size, stride=None, ceil_mode=False, data_format="NCL", name=None):
    return _w(TF.lp_pool1d(x._t, norm_type, kernel_size, stride, ceil_mode))


def lp_pool2d(x, norm_type, kernel_size, stride=None, ceil_mode=False, data_format="NCHW", name=None):
    return _w(TF.lp_pool2d(x._t, norm_type, kernel_size, stride, ceil_mode))


register_ops(globals(), __all__)
