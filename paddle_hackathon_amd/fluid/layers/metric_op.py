"""``fluid.layers.accuracy`` / ``auc`` (reference: python/paddle/fluid/layers/metric_op.py,
paddle/fluid/operators/metrics/auc_op.h)."""
from __future__ import annotations

import torch

from ._common import T, W, dev

__all__ = ["accuracy", "auc"]


def accuracy(input, label, k=1, correct=None, total=None):
    x = T(input)
    y = T(label).reshape(-1, 1).long()
    topk = torch.topk(x, k, -1).indices
    hit = (topk == y).any(-1)
    n_ok, n = int(hit.sum()), hit.numel()
    acc = W(torch.tensor([n_ok / max(n, 1)], dtype=torch.float32, device=dev()))
    if correct is not None:
        correct._t = torch.tensor([n_ok], dtype=torch.int32, device=dev())
    if total is not None:
        total._t = torch.tensor([n], dtype=torch.int32, device=dev())
    return acc


_STATE = {}


def _auc_of(pos, neg, curve):
    """trapezoid area under ROC (or PR) from per-threshold-bin positive / negative counts"""
    tp = torch.flip(torch.cumsum(torch.flip(pos, [0]), 0), [0]).double()
    fp = torch.flip(torch.cumsum(torch.flip(neg, [0]), 0), [0]).double()
    P, N = tp[0], fp[0]
    if P == 0 or N == 0:
        return 0.0
    if curve == "ROC":
        tpr = torch.cat([tp / P, torch.zeros(1, dtype=tp.dtype)])
        fpr = torch.cat([fp / N, torch.zeros(1, dtype=fp.dtype)])
        return float(((fpr[:-1] - fpr[1:]) * (tpr[:-1] + tpr[1:]) / 2).sum())
    prec = tp / (tp + fp).clamp_min(1)
    rec = tp / P
    rec2 = torch.cat([rec, torch.zeros(1, dtype=rec.dtype)])
    return float(((rec2[:-1] - rec2[1:]) * prec).sum())


def auc(input, label, curve="ROC", num_thresholds=2 ** 12 - 1, topk=1, slide_steps=1):
    """(global AUC, batch AUC, [batch_stat_pos, batch_stat_neg, stat_pos, stat_neg]); the global
    statistics accumulate over calls (the reference keeps them in persistable variables)"""
    p = T(input).float()
    p = p[:, -1] if p.dim() == 2 else p.reshape(-1)
    y = T(label).reshape(-1).long()
    bins = (p * num_thresholds).long().clamp(0, num_thresholds)
    pos = torch.bincount(bins[y == 1], minlength=num_thresholds + 1).cpu()
    neg = torch.bincount(bins[y != 1], minlength=num_thresholds + 1).cpu()
    st = _STATE.setdefault((curve, num_thresholds), {"pos": torch.zeros_like(pos), "neg": torch.zeros_like(neg)})
    st["pos"] += pos
    st["neg"] += neg
    g = _auc_of(st["pos"], st["neg"], curve)
    b = _auc_of(pos, neg, curve)
    f = lambda v: W(torch.tensor([v], dtype=torch.float64, device=dev()))  # noqa: E731
    t = lambda v: W(v.reshape(1, -1).to(dev()))  # noqa: E731
    return f(g), f(b), [t(pos), t(neg), t(st["pos"]), t(st["neg"])]
