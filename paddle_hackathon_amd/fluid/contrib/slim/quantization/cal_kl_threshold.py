"""Activation-threshold calibration (reference: python/paddle/fluid/contrib/slim/quantization/
cal_kl_threshold.py and the algo branches of post_training_quantization.py).

All calibrators see |x| statistics collected over the calibration batches:

* ``abs_max`` / ``min_max``: the largest |x| seen
* ``avg``: the mean over batches of each batch's max |x|
* ``hist``: the ``hist_percent`` quantile of the |x| histogram
* ``KL``: the histogram cut that minimises the KL divergence between the clipped distribution
  and its 2^(bits-1)-level quantization (the entropy calibration of TensorRT-style INT8)
* ``mse`` / ``emd``: the clip value (over a grid of fractions of max |x|) whose quant-dequant of the
  sampled activations has the least squared error / the least |mean| + |std| difference
"""
from __future__ import annotations

import numpy as np

__all__ = ["cal_kl_threshold", "hist_threshold", "search_threshold", "Calibrator"]


def _kl(p, q, eps=1e-4):
    """KL(p || q); bins where q has no mass but p has are smoothed with ``eps`` (they would make
    the divergence infinite — e.g. a cut whose last bin holds the clipped tail)"""
    m = p > 0
    qq = np.where(q > 0, q, eps)
    qq = qq / qq.sum()
    return float(np.sum(p[m] * np.log(p[m] / qq[m])))


def cal_kl_threshold(hist, bin_width, bits=8):
    """KL-optimal threshold of an |x| histogram (``hist`` counts of bins of ``bin_width``)"""
    hist = np.asarray(hist, dtype=np.float64)
    n_bins = len(hist)
    levels = 2 ** (bits - 1)
    if hist.sum() == 0:
        return bin_width * n_bins
    best, best_i = None, n_bins
    # candidate cuts from half the range up (as the reference's search: a cut below max|x| / 2
    # clips too much of a ReLU output whose zero bin dominates the histogram), ~160 of them;
    # a cut whose last kept bin is empty is skipped
    start = max(min(levels, n_bins), (n_bins - 1) // 2)
    stride = max(1, (n_bins - start) // 160)
    for i in list(range(start, n_bins + 1, stride)) + ([n_bins] if (n_bins - start) % stride else []):
        if hist[i - 1] == 0:
            continue
        ref = hist[:i].copy()
        ref[i - 1] += hist[i:].sum()          # clipped mass folds into the last kept bin
        if ref.sum() == 0:
            continue
        # quantize the first i bins into ``levels`` groups, spread each group evenly over its
        # non-empty bins
        edges = np.linspace(0, i, levels + 1)
        q = np.zeros(i)
        src = hist[:i]
        for j in range(levels):
            lo, hi = int(np.floor(edges[j])), int(np.ceil(edges[j + 1]))
            hi = max(hi, lo + 1)
            seg = src[lo:hi]
            nz = seg > 0
            if nz.any():
                q[lo:hi][nz] = seg.sum() / nz.sum()
        p = ref / ref.sum()
        qs = q.sum()
        if qs == 0:
            continue
        d = _kl(p, q / qs)
        if best is None or d < best:
            best, best_i = d, i
    return (best_i + 0.5) * bin_width


def hist_threshold(hist, bin_width, percent=0.99999):
    c = np.cumsum(np.asarray(hist, dtype=np.float64))
    if c[-1] == 0:
        return bin_width * len(hist)
    i = int(np.searchsorted(c / c[-1], percent))
    return (i + 1) * bin_width


def _qdq(x, s, bits):
    bn = 2 ** (bits - 1) - 1
    return np.round(np.clip(x, -s, s) / s * bn) * s / bn


def search_threshold(samples, abs_max, bits=8, algo="mse", steps=100):
    """grid search of the clip value on sampled activations (algo 'mse' | 'emd')"""
    x = np.concatenate([np.asarray(s, dtype=np.float64).ravel() for s in samples]) if samples else np.zeros(1)
    if abs_max <= 0:
        return 1e-8
    best, best_s = None, abs_max
    for k in range(1, steps + 1):
        s = abs_max * (0.3 + 0.7 * k / steps)
        y = _qdq(x, s, bits)
        if algo == "emd":
            loss = abs(float(x.mean() - y.mean())) + abs(float(x.std() - y.std()))
        else:
            loss = float(np.mean((x - y) ** 2))
        if best is None or loss < best:
            best, best_s = loss, s
    return best_s


class Calibrator:
    """per-tensor statistics of one activation over the calibration batches"""

    def __init__(self, algo="KL", bits=8, hist_percent=0.99999, bins=2048, max_samples=20):
        self.algo, self.bits, self.percent, self.bins = algo, bits, hist_percent, bins
        self.abs_max = 0.0
        self.batch_max = []
        self.samples = []
        self.max_samples = max_samples
        self._values = []

    def update(self, x):
        a = np.abs(np.asarray(x, dtype=np.float32)).ravel()
        m = float(a.max()) if a.size else 0.0
        self.abs_max = max(self.abs_max, m)
        self.batch_max.append(m)
        if self.algo in ("KL", "hist"):
            self._values.append(a)
        if self.algo in ("mse", "emd") and len(self.samples) < self.max_samples:
            self.samples.append(np.asarray(x, dtype=np.float32))

    def threshold(self):
        if self.algo in ("abs_max", "min_max"):
            return self.abs_max
        if self.algo == "avg":
            return float(np.mean(self.batch_max)) if self.batch_max else 0.0
        if self.algo in ("mse", "emd"):
            return search_threshold(self.samples, self.abs_max, self.bits, self.algo)
        if self.abs_max <= 0:
            return 0.0
        hist = np.zeros(self.bins)
        for a in self._values:
            hist += np.histogram(a, bins=self.bins, range=(0.0, self.abs_max))[0]
        width = self.abs_max / self.bins
        if self.algo == "hist":
            return hist_threshold(hist, width, self.percent)
        return min(self.abs_max, cal_kl_threshold(hist, width, self.bits))
