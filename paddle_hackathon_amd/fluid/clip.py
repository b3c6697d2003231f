"""``paddle.fluid.clip`` (reference: python/paddle/fluid/clip.py)."""
from __future__ import annotations

import torch

from ..nn.clip import ClipGradByValue, ClipGradByNorm, ClipGradByGlobalNorm  # noqa: F401

__all__ = ["set_gradient_clip", "ErrorClipByValue", "ClipGradByValue", "ClipGradByNorm", "ClipGradByGlobalNorm"]

_GLOBAL_CLIP = {"clip": None, "params": None}


def set_gradient_clip(clip, param_list=None, program=None):
    """default gradient clip for optimizers built without ``grad_clip`` (static-graph API)"""
    _GLOBAL_CLIP["clip"] = clip
    _GLOBAL_CLIP["params"] = param_list


class ErrorClipByValue:
    """clips the gradient flowing back through a variable to [min, max]"""

    def __init__(self, max, min=None):
        self.max = float(max)
        self.min = -self.max if min is None else float(min)

    def __call__(self, grad):
        return grad.clamp(self.min, self.max) if isinstance(grad, torch.Tensor) else grad

    def attach(self, var):
        t = var._t
        if t.requires_grad:
            t.register_hook(self)
        return var

# 1.x names (reference: fluid/clip.py)
GradientClipByGlobalNorm = ClipGradByGlobalNorm
GradientClipByNorm = ClipGradByNorm
GradientClipByValue = ClipGradByValue
