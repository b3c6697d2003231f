"""Loss layers (reference: python/paddle/nn/layer/loss.py)."""
from __future__ import annotations

from .. import functional as F
from .. import initializer as I
from .layers import Layer

__all__ = ["BCEWithLogitsLoss", "CrossEntropyLoss", "HSigmoidLoss", "MSELoss", "L1Loss", "NLLLoss", "BCELoss",
           "KLDivLoss", "MarginRankingLoss", "CTCLoss", "SmoothL1Loss", "HingeEmbeddingLoss", "CosineEmbeddingLoss",
           "TripletMarginLoss", "TripletMarginWithDistanceLoss", "MultiLabelSoftMarginLoss", "SoftMarginLoss"]


class BCEWithLogitsLoss(Layer):
    def __init__(self, weight=None, reduction="mean", pos_weight=None, name=None):
        super().__init__()
        self.weight, self.reduction, self.pos_weight = weight, reduction, pos_weight

    def forward(self, logit, label):
        return F.binary_cross_entropy_with_logits(logit, label, self.weight, self.reduction, self.pos_weight)


class CrossEntropyLoss(Layer):
    def __init__(self, weight=None, ignore_index=-100, reduction="mean", soft_label=False, axis=-1,
                 use_softmax=True, name=None, label_smoothing=0.0):
        super().__init__()
        self.weight, self.ignore_index, self.reduction = weight, ignore_index, reduction
        self.soft_label, self.axis, self.use_softmax = soft_label, axis, use_softmax
        self.label_smoothing = label_smoothing

    def forward(self, input, label):
        return F.cross_entropy(input, label, self.weight, self.ignore_index, self.reduction, self.soft_label,
                               self.axis, self.use_softmax, label_smoothing=self.label_smoothing)


class HSigmoidLoss(Layer):
    def __init__(self, feature_size, num_classes, weight_attr=None, bias_attr=None, is_custom=False, is_sparse=False, name=None):
        super().__init__()
        self._num_classes = num_classes
        self.weight = self.create_parameter([num_classes - 1, feature_size], attr=weight_attr)
        self.bias = self.create_parameter([num_classes - 1, 1], attr=bias_attr, is_bias=True)

    def forward(self, input, label, path_table=None, path_code=None):
        return F.hsigmoid_loss(input, label, self._num_classes, self.weight, self.bias, path_table, path_code)


def _simple(name, fn, params):
    def __init__(self, *args, **kwargs):
        Layer.__init__(self)
        vals = dict(params)
        for k, v in zip(params, args):
            vals[k] = v
        for k, v in kwargs.items():
            if k != "name":
                vals[k] = v
        self._kw = vals

    def forward(self, *inputs):
        return fn(*inputs, **self._kw)

    return type(name, (Layer,), {"__init__": __init__, "forward": forward})


MSELoss = _simple("MSELoss", F.mse_loss, {"reduction": "mean"})
L1Loss = _simple("L1Loss", F.l1_loss, {"reduction": "mean"})
NLLLoss = _simple("NLLLoss", F.nll_loss, {"weight": None, "ignore_index": -100, "reduction": "mean"})
BCELoss = _simple("BCELoss", F.binary_cross_entropy, {"weight": None, "reduction": "mean"})
KLDivLoss = _simple("KLDivLoss", F.kl_div, {"reduction": "mean"})
MarginRankingLoss = _simple("MarginRankingLoss", F.margin_ranking_loss, {"margin": 0.0, "reduction": "mean"})
SmoothL1Loss = _simple("SmoothL1Loss", F.smooth_l1_loss, {"reduction": "mean", "delta": 1.0})
HingeEmbeddingLoss = _simple("HingeEmbeddingLoss", F.hinge_embedding_loss, {"margin": 1.0, "reduction": "mean"})
CosineEmbeddingLoss = _simple("CosineEmbeddingLoss", F.cosine_embedding_loss, {"margin": 0, "reduction": "mean"})
TripletMarginLoss = _simple("TripletMarginLoss", F.triplet_margin_loss,
                            {"margin": 1.0, "p": 2.0, "epsilon": 1e-6, "swap": False, "reduction": "mean"})
TripletMarginWithDistanceLoss = _simple("TripletMarginWithDistanceLoss", F.triplet_margin_with_distance_loss,
                                        {"distance_function": None, "margin": 1.0, "swap": False, "reduction": "mean"})
MultiLabelSoftMarginLoss = _simple("MultiLabelSoftMarginLoss", F.multi_label_soft_margin_loss, {"weight": None, "reduction": "mean"})
SoftMarginLoss = _simple("SoftMarginLoss", F.soft_margin_loss, {"reduction": "mean"})


class CTCLoss(Layer):
    def __init__(self, blank=0, reduction="mean"):
        super().__init__()
        self.blank, self.reduction = blank, reduction

    def forward(self, log_probs, labels, input_lengths, label_lengths, norm_by_times=False):
        return F.ctc_loss(log_probs, labels, input_lengths, label_lengths, self.blank, self.reduction, norm_by_times)
