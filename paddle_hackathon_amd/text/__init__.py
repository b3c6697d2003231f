"""``paddle.text`` (reference: python/paddle/text/{viterbi_decode.py,datasets/*}).

Datasets read the reference's on-disk formats from ``data_file`` / the local cache when
present; with no network they fall back to deterministic synthetic corpora of the same
structure (documented per class), so pipelines and tests run offline."""
from __future__ import annotations

import torch

from ..framework.core import Tensor, _wrap
from ..framework.dispatch import register_ops
from ..nn.layer.layers import Layer
from .datasets import Conll05st, Imdb, Imikolov, Movielens, UCIHousing, WMT14, WMT16  # noqa: F401
from . import datasets  # noqa: F401

__all__ = ["Conll05st", "Imdb", "Imikolov", "Movielens", "UCIHousing", "WMT14", "WMT16", "ViterbiDecoder",
           "viterbi_decode"]


def viterbi_decode(potentials, transition_params, lengths, include_bos_eos_tag=True, name=None):
    """Batched Viterbi (reference: phi/kernels/cpu/viterbi_decode_kernel.cc). With
    ``include_bos_eos_tag`` row N-1 of the transitions is the start tag and row N-2 the stop tag.
    Returns (scores [B], path [B, max(lengths)])."""
    x = potentials._t
    trans = transition_params._t.to(x.dtype)
    length = lengths._t.long().reshape(-1).to(x.device)
    B, T, N = x.shape
    max_len = int(length.max().item()) if B else 0
    stop, start = trans[N - 2], trans[N - 1]
    alpha = x[:, 0]
    left = length - 1
    if include_bos_eos_tag:
        alpha = alpha + start + stop * (left == 0).to(x.dtype)[:, None]
    hist = []
    for i in range(1, max_len):
        s = alpha[:, :, None] + trans[None]
        amax, arg = s.max(1)
        hist.append(arg)
        nxt = amax + x[:, i]
        m = (left > 0).to(x.dtype)[:, None]
        alpha = nxt * m + alpha * (1 - m)
        if include_bos_eos_tag:
            alpha = alpha + stop * (left == 1).to(x.dtype)[:, None]
        left = left - 1
    scores, last = alpha.max(1)
    actual = min(T, max_len)
    path = torch.zeros(max_len, B, dtype=torch.int64, device=x.device)
    if actual > 0:
        path[actual - 1] = last * (left >= 0).long()
    k = 1
    for h in reversed(hist):
        k += 1
        left = left + 1
        upd = h.gather(1, last[:, None]).squeeze(1) * (left > 0).long()
        zl = (left == 0).long()
        upd = upd * (1 - zl) + last * zl
        path[actual - k] = upd
        last = upd + last * (left < 0).long()
    return _wrap(scores), _wrap(path.t().contiguous())


class ViterbiDecoder(Layer):
    def __init__(self, transitions, include_bos_eos_tag=True, name=None):
        super().__init__()
        self.transitions = transitions
        self.include_bos_eos_tag = include_bos_eos_tag

    def forward(self, potentials, lengths):
        return viterbi_decode(potentials, self.transitions, lengths, self.include_bos_eos_tag)


register_ops(globals(), ["viterbi_decode"])
