"""PTQ quantizers (reference: fluid/contrib/slim/quantization/imperative/ptq_quantizer.py): each
samples the tensors a hooked layer sees during calibration and turns them into thresholds.

* ``AbsmaxQuantizer`` — max |x| per tensor
* ``PerChannelAbsmaxQuantizer`` — weights: max |w| per output channel (conv axis 0, linear 1)
* ``HistQuantizer`` — the ``hist_percent`` quantile of an |x| histogram (grown by re-binning)
* ``KLQuantizer`` — the KL-optimal cut of that histogram (cal_kl_threshold)
"""
from __future__ import annotations

import abc

import numpy as np

from ..cal_kl_threshold import cal_kl_threshold, hist_threshold

__all__ = ["BaseQuantizer", "AbsmaxQuantizer", "PerChannelAbsmaxQuantizer", "KLQuantizer", "HistQuantizer",
           "SUPPORT_ACT_QUANTIZERS", "SUPPORT_WT_QUANTIZERS"]


def _np(t):
    if hasattr(t, "numpy"):
        return np.asarray(t.numpy(), dtype=np.float32)
    return np.asarray(t, dtype=np.float32)


class BaseQuantizer(metaclass=abc.ABCMeta):
    def __init__(self, quant_bits=8):
        assert isinstance(quant_bits, int) and 0 < quant_bits <= 16
        self.quant_bits = quant_bits
        self.thresholds = []
        self.abs_max_vals = []

    @abc.abstractmethod
    def sample_data(self, layer, tensors):
        pass

    @abc.abstractmethod
    def cal_thresholds(self):
        pass


class AbsmaxQuantizer(BaseQuantizer):
    def sample_data(self, layer, tensors):
        vals = [float(np.abs(_np(t)).max()) if _np(t).size else 0.0 for t in tensors]
        self.abs_max_vals = vals if not self.abs_max_vals else [max(a, b) for a, b in zip(self.abs_max_vals, vals)]

    def cal_thresholds(self):
        self.thresholds = list(self.abs_max_vals)


class PerChannelAbsmaxQuantizer(BaseQuantizer):
    def sample_data(self, layer, tensors):
        from ......nn import Conv2DTranspose, Linear
        axis = 1 if isinstance(layer, (Linear, Conv2DTranspose)) else 0
        vals = []
        for t in tensors:
            a = np.abs(_np(t))
            vals.append(np.moveaxis(a, axis, 0).reshape(a.shape[axis], -1).max(axis=1))
        self.abs_max_vals = vals if not self.abs_max_vals else [np.maximum(a, b) for a, b in
                                                                 zip(self.abs_max_vals, vals)]

    def cal_thresholds(self):
        self.thresholds = [np.asarray(v, dtype=np.float32) for v in self.abs_max_vals]


class BaseHistQuantizer(BaseQuantizer, metaclass=abc.ABCMeta):
    def __init__(self, quant_bits=8, bins=1024, upsample_bins=64):
        super().__init__(quant_bits)
        self.bins, self.upsample_bins = bins, upsample_bins
        self.hists = []

    def sample_data(self, layer, tensors):
        arrs = [np.abs(_np(t)).ravel() for t in tensors]
        if not self.hists:
            self.abs_max_vals = [float(a.max()) if a.size else 0.0 for a in arrs]
            self.hists = [np.histogram(a, bins=self.bins, range=(0.0, m if m > 0 else 1.0))[0].astype(np.float64)
                          for a, m in zip(arrs, self.abs_max_vals)]
            return
        for i, a in enumerate(arrs):
            m = float(a.max()) if a.size else 0.0
            old = self.abs_max_vals[i]
            if m > old:   # widen: re-bin the old histogram onto the new range (upsampled)
                up = np.repeat(self.hists[i] / self.upsample_bins, self.upsample_bins)
                centers = (np.arange(len(up)) + 0.5) * (old / len(up))
                self.hists[i] = np.histogram(centers, bins=self.bins, range=(0.0, m), weights=up)[0]
                self.abs_max_vals[i] = m
            rng = self.abs_max_vals[i] if self.abs_max_vals[i] > 0 else 1.0
            self.hists[i] += np.histogram(a, bins=self.bins, range=(0.0, rng))[0]


class HistQuantizer(BaseHistQuantizer):
    def __init__(self, quant_bits=8, bins=1024, upsample_bins=64, hist_percent=0.99999):
        super().__init__(quant_bits, bins, upsample_bins)
        self.hist_percent = hist_percent

    def cal_thresholds(self):
        self.thresholds = [hist_threshold(h, (m if m > 0 else 1.0) / self.bins, self.hist_percent)
                           for h, m in zip(self.hists, self.abs_max_vals)]


class KLQuantizer(BaseHistQuantizer):
    def cal_thresholds(self):
        self.thresholds = [min(m, cal_kl_threshold(h, (m if m > 0 else 1.0) / self.bins, self.quant_bits))
                           for h, m in zip(self.hists, self.abs_max_vals)]


SUPPORT_ACT_QUANTIZERS = [AbsmaxQuantizer, HistQuantizer, KLQuantizer]
SUPPORT_WT_QUANTIZERS = [AbsmaxQuantizer, PerChannelAbsmaxQuantizer]
