"""``paddle.signal`` stft/istft (reference: python/paddle/signal.py)."""
from __future__ import annotations

import torch

from .framework.core import _wrap, _unwrap
from .framework.dispatch import register_ops

__all__ = ["stft", "istft", "frame", "overlap_add"]


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


def frame(x, frame_length, hop_length, axis=-1, name=None):
    """frames of ``frame_length`` every ``hop_length`` samples along the first or last axis
    (reference: signal.py frame): axis=-1: [..., T] -> [..., frame_length, num_frames];
    axis=0: [T, ...] -> [num_frames, frame_length, ...]"""
    t = x._t
    if axis not in (0, -1, t.dim() - 1):
        raise ValueError("frame: axis must be 0 or -1")
    if frame_length > t.shape[axis]:
        raise ValueError("frame: frame_length exceeds the sequence length")
    if axis == 0:
        u = t.unfold(0, frame_length, hop_length)          # [num, ..., frame]
        return _wrap(u.movedim(-1, 1).contiguous())
    u = t.unfold(-1, frame_length, hop_length)             # [..., num, frame]
    return _wrap(u.transpose(-1, -2).contiguous())


def overlap_add(x, hop_length, axis=-1, name=None):
    """the sum of overlapping frames (reference: signal.py overlap_add, the inverse layout of
    ``frame``): axis=-1: [..., frame_length, num_frames] -> [..., (num - 1) * hop + frame_length];
    axis=0: [num_frames, frame_length, ...] -> [(num - 1) * hop + frame_length, ...]"""
    t = x._t
    if axis == 0:
        t = t.movedim(0, -1).movedim(0, -2)                # -> [..., frame_length, num_frames]
    fl, nf = t.shape[-2], t.shape[-1]
    n = (nf - 1) * hop_length + fl
    lead = t.shape[:-2]
    flat = t.reshape(-1, fl, nf)
    out = torch.nn.functional.fold(flat, output_size=(1, n), kernel_size=(1, fl), stride=(1, hop_length))
    out = out.reshape(*lead, n)
    if axis == 0:
        out = out.movedim(-1, 0)
    return _wrap(out)


register_ops(globals(), ["frame", "overlap_add"])
