"""``paddle.fft`` (reference: python/paddle/fft.py). Transforms run on rocFFT through
PyTorch-ROCm; ``norm`` follows Paddle's "backward"|"ortho"|"forward" convention."""
from __future__ import annotations

import torch

from .framework.core import _wrap, _unwrap
from .framework.dispatch import register_ops
from .tensor._helpers import _axis, _int_list

__all__ = ["fft", "fft2", "fftn", "ifft", "ifft2", "ifftn", "rfft", "rfft2", "rfftn", "irfft", "irfft2", "irfftn",
           "hfft", "hfft2", "hfftn", "ihfft", "ihfft2", "ihfftn", "fftfreq", "rfftfreq", "fftshift", "ifftshift"]


def _check_norm(norm):
    if norm not in ("backward", "ortho", "forward"):
        raise ValueError(f"Unexpected norm: {norm}. Norm should be forward, backward or ortho")
    return norm


def _one(fn):
    def op(x, n=None, axis=-1, norm="backward", name=None):
        return _wrap(fn(_unwrap(x), n=n, dim=axis, norm=_check_norm(norm)))
    op.__name__ = fn.__name__
    return op


def _many(fn, default_axes):
    def op(x, s=None, axes=default_axes, norm="backward", name=None):
        dims = _axis(axes)
        if isinstance(dims, int):
            dims = (dims,)
        return _wrap(fn(_unwrap(x), s=_int_list(s), dim=dims, norm=_check_norm(norm)))
    op.__name__ = fn.__name__
    return op


fft, ifft, rfft, irfft, hfft, ihfft = (_one(f) for f in (torch.fft.fft, torch.fft.ifft, torch.fft.rfft,
                                                          torch.fft.irfft, torch.fft.hfft, torch.fft.ihfft))
fft2, ifft2, rfft2, irfft2, hfft2, ihfft2 = (_many(f, (-2, -1)) for f in (
    torch.fft.fftn, torch.fft.ifftn, torch.fft.rfftn, torch.fft.irfftn, torch.fft.hfftn, torch.fft.ihfftn))
fftn, ifftn, rfftn, irfftn, hfftn, ihfftn = (_many(f, None) for f in (
    torch.fft.fftn, torch.fft.ifftn, torch.fft.rfftn, torch.fft.irfftn, torch.fft.hfftn, torch.fft.ihfftn))
for _n in __all__[:18]:
    globals()[_n].__name__ = _n


def fftfreq(n, d=1.0, dtype=None, name=None):
    from .framework.core import convert_dtype, default_device
    return _wrap(torch.fft.fftfreq(n, d, dtype=convert_dtype(dtype) if dtype else torch.float32,
                                   device=default_device()))


def rfftfreq(n, d=1.0, dtype=None, name=None):
    from .framework.core import convert_dtype, default_device
    return _wrap(torch.fft.rfftfreq(n, d, dtype=convert_dtype(dtype) if dtype else torch.float32,
                                    device=default_device()))


def fftshift(x, axes=None, name=None):
    return _wrap(torch.fft.fftshift(_unwrap(x), dim=_axis(axes)))


def ifftshift(x, axes=None, name=None):
    return _wrap(torch.fft.ifftshift(_unwrap(x), dim=_axis(axes)))


register_ops(globals(), __all__)
