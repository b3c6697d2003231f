"""``paddle.metric`` (reference: python/paddle/metric/metrics.py)."""
from __future__ import annotations

import abc

import numpy as np
import torch

from ..framework.core import Tensor, _wrap
from ..framework.dispatch import register_ops

__all__ = ["Metric", "Accuracy", "Precision", "Recall", "Auc", "accuracy"]


def _np(x):
    if isinstance(x, Tensor):
        return x.numpy()
    return np.asarray(x)


class Metric(abc.ABC):
    def __init__(self):
        pass

    @abc.abstractmethod
    def reset(self):
        raise NotImplementedError

    @abc.abstractmethod
    def update(self, *args):
        raise NotImplementedError

    @abc.abstractmethod
    def accumulate(self):
        raise NotImplementedError

    @abc.abstractmethod
    def name(self):
        raise NotImplementedError

    def compute(self, *args):
        return args


class Accuracy(Metric):
    def __init__(self, topk=(1,), name=None, *args, **kwargs):
        super().__init__()
        self.topk = topk
        self.maxk = max(topk)
        self._init_name(name)
        self.reset()

    def compute(self, pred, label, *args):
        p = pred._t if isinstance(pred, Tensor) else torch.as_tensor(np.asarray(pred))
        l = label._t if isinstance(label, Tensor) else torch.as_tensor(np.asarray(label))
        idx = torch.argsort(p, dim=-1, descending=True)[..., : self.maxk]
        if l.dim() == 1 or (l.dim() == 2 and l.shape[-1] == 1):
            l = l.reshape(-1, 1)
        elif l.shape[-1] != 1:
            l = torch.argmax(l, -1, keepdim=True)
        return _wrap((idx == l.to(idx.device)).float())

    def update(self, correct, *args):
        c = _np(correct)
        accs = []
        for i, k in enumerate(self.topk):
            num_corrects = c[..., :k].sum()
            num_samples = int(np.prod(c.shape[:-1]))
            accs.append(float(num_corrects) / num_samples)
            self.total[i] += num_corrects
            self.count[i] += num_samples
        return accs[0] if len(self.topk) == 1 else accs

    def reset(self):
        self.total = [0.0] * len(self.topk)
        self.count = [0] * len(self.topk)

    def accumulate(self):
        res = [float(t) / c if c > 0 else 0.0 for t, c in zip(self.total, self.count)]
        return res[0] if len(self.topk) == 1 else res

    def _init_name(self, name):
        name = name or "acc"
        self._name = [f"{name}_top{k}" for k in self.topk] if self.maxk != 1 else [name]

    def name(self):
        return self._name


class Precision(Metric):
    def __init__(self, name="precision", *args, **kwargs):
        super().__init__()
        self.tp = self.fp = 0
        self._name = name

    def update(self, preds, labels):
        p = np.rint(_np(preds)).astype("int32").reshape(-1)
        l = _np(labels).astype("int32").reshape(-1)
        self.tp += int(((p == 1) & (l == 1)).sum())
        self.fp += int(((p == 1) & (l == 0)).sum())

    def reset(self):
        self.tp = self.fp = 0

    def accumulate(self):
        ap = self.tp + self.fp
        return float(self.tp) / ap if ap != 0 else 0.0

    def name(self):
        return self._name


class Recall(Metric):
    def __init__(self, name="recall", *args, **kwargs):
        super().__init__()
        self.tp = self.fn = 0
        self._name = name

    def update(self, preds, labels):
        p = np.rint(_np(preds)).astype("int32").reshape(-1)
        l = _np(labels).astype("int32").reshape(-1)
        self.tp += int(((p == 1) & (l == 1)).sum())
        self.fn += int(((p == 0) & (l == 1)).sum())

    def reset(self):
        self.tp = self.fn = 0

    def accumulate(self):
        r = self.tp + self.fn
        return float(self.tp) / r if r != 0 else 0.0

    def name(self):
        return self._name


class Auc(Metric):
    def __init__(self, curve="ROC", num_thresholds=4095, name="auc", *args, **kwargs):
        super().__init__()
        self._curve, self._num_thresholds, self._name = curve, num_thresholds, name
        self.reset()

    def update(self, preds, labels):
        p = _np(preds)
        l = _np(labels).reshape(-1)
        pos_prob = p[:, 1] if p.ndim == 2 and p.shape[1] == 2 else p.reshape(-1)
        bins = np.clip((pos_prob * self._num_thresholds).astype("int64"), 0, self._num_thresholds)
        np.add.at(self._stat_pos, bins[l == 1], 1)
        np.add.at(self._stat_neg, bins[l != 1], 1)

    def reset(self):
        self._stat_pos = np.zeros(self._num_thresholds + 1, dtype="int64")
        self._stat_neg = np.zeros(self._num_thresholds + 1, dtype="int64")

    @staticmethod
    def trapezoid_area(x1, x2, y1, y2):
        return abs(x1 - x2) * (y1 + y2) / 2.0

    def accumulate(self):
        tot_pos = tot_neg = 0.0
        auc = 0.0
        idx = self._num_thresholds
        while idx >= 0:
            tp_prev, tn_prev = tot_pos, tot_neg
            tot_pos += self._stat_pos[idx]
            tot_neg += self._stat_neg[idx]
            auc += self.trapezoid_area(tot_neg, tn_prev, tot_pos, tp_prev)
            idx -= 1
        return auc / tot_pos / tot_neg if tot_pos > 0 and tot_neg > 0 else 0.0

    def name(self):
        return self._name


def accuracy(input, label, k=1, correct=None, total=None, name=None):
    p, l = input._t, label._t
    topk = torch.topk(p, k, -1).indices
    l = l.reshape(-1, 1)
    c = (topk == l).any(-1).float().sum()
    n = torch.tensor(float(p.shape[0]), device=p.device)
    if correct is not None:
        correct._t = c.to(torch.int32)
    if total is not None:
        total._t = n.to(torch.int32)
    return _wrap(c / n)


register_ops(globals(), ["accuracy"])
