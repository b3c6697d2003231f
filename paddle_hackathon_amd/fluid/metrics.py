"""``paddle.fluid.metrics`` (reference: python/paddle/fluid/metrics.py): host-side streaming
metrics over numpy batches."""
from __future__ import annotations

import copy

import numpy as np

__all__ = ["MetricBase", "CompositeMetric", "Precision", "Recall", "Accuracy", "ChunkEvaluator", "EditDistance",
           "DetectionMAP", "Auc"]


def _np(x):
    return x.numpy() if hasattr(x, "numpy") else np.asarray(x)


class MetricBase:
    def __init__(self, name):
        self._name = str(name) if name is not None else type(self).__name__

    def __str__(self):
        return self._name

    def reset(self):
        for k, v in list(self.__dict__.items()):
            if k.startswith("_"):
                continue
            if isinstance(v, (int, float)):
                setattr(self, k, 0)
            elif isinstance(v, np.ndarray):
                setattr(self, k, np.zeros_like(v))
            else:
                setattr(self, k, None)

    def get_config(self):
        return {"name": self._name, "states": copy.deepcopy({k: v for k, v in self.__dict__.items()
                                                               if not k.startswith("_")})}

    def update(self, preds, labels):
        raise NotImplementedError

    def eval(self):
        raise NotImplementedError


class CompositeMetric(MetricBase):
    def __init__(self, name=None):
        super().__init__(name)
        self._metrics = []

    def add_metric(self, metric):
        if not isinstance(metric, MetricBase):
            raise ValueError("SubMetric should be inherit from MetricBase.")
        self._metrics.append(metric)

    def update(self, preds, labels):
        for m in self._metrics:
            m.update(preds, labels)

    def eval(self):
        return [m.eval() for m in self._metrics]


class Precision(MetricBase):
    """binary precision: predictions are rounded to 0 / 1"""

    def __init__(self, name=None):
        super().__init__(name)
        self.tp = 0
        self.fp = 0

    def update(self, preds, labels):
        p = np.rint(_np(preds)).astype("int32").reshape(-1)
        y = _np(labels).astype("int32").reshape(-1)
        self.tp += int(((p == 1) & (y == 1)).sum())
        self.fp += int(((p == 1) & (y != 1)).sum())

    def eval(self):
        ap = self.tp + self.fp
        return float(self.tp) / ap if ap != 0 else 0.0


class Recall(MetricBase):
    def __init__(self, name=None):
        super().__init__(name)
        self.tp = 0
        self.fn = 0

    def update(self, preds, labels):
        p = np.rint(_np(preds)).astype("int32").reshape(-1)
        y = _np(labels).astype("int32").reshape(-1)
        self.tp += int(((p == 1) & (y == 1)).sum())
        self.fn += int(((p != 1) & (y == 1)).sum())

    def eval(self):
        r = self.tp + self.fn
        return float(self.tp) / r if r != 0 else 0.0


class Accuracy(MetricBase):
    """weighted running mean of per-batch accuracies"""

    def __init__(self, name=None):
        super().__init__(name)
        self.value = 0.0
        self.weight = 0.0

    def update(self, value, weight):
        self.value += float(np.asarray(_np(value)).reshape(-1)[0]) * float(weight)
        self.weight += float(weight)

    def eval(self):
        if self.weight == 0:
            raise ValueError("There is no data in Accuracy Metrics. Please check layers.accuracy output has added "
                             "to Accuracy.")
        return self.value / self.weight


class ChunkEvaluator(MetricBase):
    def __init__(self, name=None):
        super().__init__(name)
        self.num_infer_chunks = 0
        self.num_label_chunks = 0
        self.num_correct_chunks = 0

    def update(self, num_infer_chunks, num_label_chunks, num_correct_chunks):
        self.num_infer_chunks += int(np.asarray(_np(num_infer_chunks)).reshape(-1)[0])
        self.num_label_chunks += int(np.asarray(_np(num_label_chunks)).reshape(-1)[0])
        self.num_correct_chunks += int(np.asarray(_np(num_correct_chunks)).reshape(-1)[0])

    def eval(self):
        p = float(self.num_correct_chunks) / self.num_infer_chunks if self.num_infer_chunks else 0.0
        r = float(self.num_correct_chunks) / self.num_label_chunks if self.num_label_chunks else 0.0
        f1 = float(2 * p * r) / (p + r) if self.num_correct_chunks else 0.0
        return p, r, f1


class EditDistance(MetricBase):
    def __init__(self, name=None):
        super().__init__(name)
        self.total_distance = 0.0
        self.seq_num = 0
        self.instance_error = 0

    def update(self, distances, seq_num):
        d = _np(distances).reshape(-1)
        n = int(np.asarray(_np(seq_num)).reshape(-1)[0])
        self.seq_num += n
        self.instance_error += int((d > 0).sum())
        self.total_distance += float(d.sum())

    def eval(self):
        if self.seq_num == 0:
            raise ValueError("There is no data in EditDistance Metric.")
        return self.total_distance / self.seq_num, self.instance_error / float(self.seq_num)


class Auc(MetricBase):
    def __init__(self, name=None, curve="ROC", num_thresholds=4095):
        super().__init__(name)
        self._curve, self._num_thresholds = curve, num_thresholds
        self._stat_pos = np.zeros(num_thresholds + 1, dtype="int64")
        self._stat_neg = np.zeros(num_thresholds + 1, dtype="int64")

    def reset(self):
        self._stat_pos[:] = 0
        self._stat_neg[:] = 0

    def update(self, preds, labels):
        p = _np(preds)
        p = p[:, -1] if p.ndim == 2 else p.reshape(-1)
        y = _np(labels).reshape(-1)
        idx = np.clip((p * self._num_thresholds).astype("int64"), 0, self._num_thresholds)
        np.add.at(self._stat_pos, idx[y == 1], 1)
        np.add.at(self._stat_neg, idx[y != 1], 1)

    def eval(self):
        tot_pos = tot_neg = 0.0
        auc = 0.0
        for i in range(self._num_thresholds, -1, -1):
            pp, nn = tot_pos, tot_neg
            tot_pos += self._stat_pos[i]
            tot_neg += self._stat_neg[i]
            auc += (tot_neg - nn) * (tot_pos + pp) / 2.0
        return auc / tot_pos / tot_neg if tot_pos > 0 and tot_neg > 0 else 0.0


def _ap(tp_list, fp_list, n_pos, version):
    if n_pos == 0:
        return None
    order = sorted(range(len(tp_list)), key=lambda i: -tp_list[i][0])
    tp = np.cumsum([tp_list[i][1] for i in order]) if order else np.zeros(0)
    fp = np.cumsum([fp_list[i][1] for i in order]) if order else np.zeros(0)
    rec = tp / n_pos
    prec = tp / np.maximum(tp + fp, 1e-12)
    if version == "11point":
        ap = 0.0
        for t in np.linspace(0, 1, 11):
            ps = prec[rec >= t]
            ap += (ps.max() if ps.size else 0.0) / 11
        return ap
    ap, prev_r = 0.0, 0.0
    for r, p in zip(rec, prec):
        if r != prev_r:
            ap += p * abs(r - prev_r)
            prev_r = r
    return ap


class DetectionMAP(MetricBase):
    """mean average precision of detections ([label, score, x1, y1, x2, y2] rows per image)
    against ground truth, 11-point or integral AP (detection_map_op.h)"""

    def __init__(self, input=None, gt_label=None, gt_box=None, gt_difficult=None, class_num=None,
                 background_label=0, overlap_threshold=0.5, evaluate_difficult=True, ap_version="integral",
                 name=None):
        super().__init__(name)
        self.class_num, self.background = class_num, background_label
        self.thr, self.eval_diff, self.version = overlap_threshold, evaluate_difficult, ap_version
        self._reset_state()

    def _reset_state(self):
        self._tp, self._fp, self._npos = {}, {}, {}

    def reset(self, executor=None, reset_program=None):
        self._reset_state()

    @staticmethod
    def _iou(a, b):
        x1, y1 = max(a[0], b[0]), max(a[1], b[1])
        x2, y2 = min(a[2], b[2]), min(a[3], b[3])
        inter = max(x2 - x1, 0.0) * max(y2 - y1, 0.0)
        u = (a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - inter
        return inter / u if u > 0 else 0.0

    def update(self, detections, gts):
        """``detections``: per image list of (label, score, box); ``gts``: per image list of
        (label, box, difficult)"""
        batch = {}
        for dets, g in zip(detections, gts):
            for lab, box, diff in g:
                if diff and not self.eval_diff:
                    continue
                self._npos[lab] = self._npos.get(lab, 0) + 1
            used = [False] * len(g)
            for lab, score, box in sorted(dets, key=lambda d: -d[1]):
                best, bi = 0.0, -1
                for j, (gl, gb, gd) in enumerate(g):
                    if gl == lab:
                        o = self._iou(box, gb)
                        if o > best:
                            best, bi = o, j
                tp = best > self.thr and bi >= 0 and not used[bi]
                if tp and g[bi][2] and not self.eval_diff:
                    continue
                if tp:
                    used[bi] = True
                self._tp.setdefault(lab, []).append((score, 1 if tp else 0))
                self._fp.setdefault(lab, []).append((score, 0 if tp else 1))
                batch[lab] = True
        return self.eval()

    def eval(self):
        aps = []
        for lab, n in self._npos.items():
            if lab == self.background:
                continue
            ap = _ap(self._tp.get(lab, []), self._fp.get(lab, []), n, self.version)
            if ap is not None:
                aps.append(ap)
        return float(np.mean(aps)) if aps else 0.0

    def get_map_var(self):
        return self.eval(), self.eval()
