"""PTQ configuration (reference: imperative/ptq_config.py)."""
from __future__ import annotations

import copy

from .ptq_quantizer import SUPPORT_ACT_QUANTIZERS, SUPPORT_WT_QUANTIZERS, BaseQuantizer, KLQuantizer, \
    PerChannelAbsmaxQuantizer

__all__ = ["PTQConfig", "default_ptq_config"]


class PTQConfig:
    """how a quantizable layer's inputs (activation_quantizer) and weights (weight_quantizer) are
    calibrated"""

    def __init__(self, activation_quantizer, weight_quantizer):
        assert isinstance(activation_quantizer, tuple(SUPPORT_ACT_QUANTIZERS))
        assert isinstance(weight_quantizer, tuple(SUPPORT_WT_QUANTIZERS))
        self.in_act_quantizer = copy.deepcopy(activation_quantizer)
        self.out_act_quantizer = copy.deepcopy(activation_quantizer)
        self.wt_quantizer = copy.deepcopy(weight_quantizer)
        self.quant_hook_handle = None
        self.enable_in_act_quantizer = False


default_ptq_config = PTQConfig(KLQuantizer(), PerChannelAbsmaxQuantizer())
