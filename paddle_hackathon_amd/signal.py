"""``paddle.signal`` stft/istft (reference: python/paddle/signal.py)."""
from __future__ import annotations

import torch

from .framework.core import _wrap, _unwrap
from .framework.dispatch import register_ops

__all__ = ["stft", "istft"]


def stft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, pad_mode="reflect",
         normalized=False, onesided=True, name=None):
    t = _unwrap(x)
    win = _unwrap(window) if window is not None else None
    if not t.is_complex() and not onesided:
        t = t.to(torch.complex64 if t.dtype != torch.float64 else torch.complex128)
    return _wrap(torch.stft(t, n_fft, hop_length=hop_length, win_length=win_length, window=win, center=center,
                            pad_mode=pad_mode, normalized=normalized, onesided=onesided if not t.is_complex() else False,
                            return_complex=True))


def istft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, normalized=False, onesided=True,
          length=None, return_complex=False, name=None):
    win = _unwrap(window) if window is not None else None
    return _wrap(torch.istft(_unwrap(x), n_fft, hop_length=hop_length, win_length=win_length, window=win,
                             center=center, normalized=normalized, onesided=onesided, length=length,
                             return_complex=return_complex))


register_ops(globals(), __all__)
