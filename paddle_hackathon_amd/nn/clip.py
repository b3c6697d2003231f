"""Gradient clipping (reference: python/paddle/fluid/clip.py).

``ClipGradByGlobalNorm`` computes the global norm with one multi-tensor HIP
reduction (ops.global_norm_sq) and scales all grads in place; under tensor /
pipeline parallelism the squared norm is all-reduced across the model-parallel
groups first (set ``_mp_group``), matching HybridParallelClipGrad.
"""
from __future__ import annotations

import torch

from ..framework.core import Tensor, _wrap
from .. import ops as _ops

__all__ = ["ClipGradByValue", "ClipGradByNorm", "ClipGradByGlobalNorm", "clip_grad_norm_", "clip_grad_value_"]


class ClipGradBase:
    def __call__(self, params_grads):
        return self._dygraph_clip(params_grads)


class ClipGradByValue(ClipGradBase):
    def __init__(self, max, min=None):
        self.max = float(max)
        self.min = -self.max if min is None else float(min)

    def _dygraph_clip(self, params_grads):
        out = []
        for p, g in params_grads:
            if g is None or not getattr(p, "need_clip", True):
                out.append((p, g))
                continue
            g._t.clamp_(self.min, self.max)
            out.append((p, g))
        return out


class ClipGradByNorm(ClipGradBase):
    def __init__(self, clip_norm):
        self.clip_norm = float(clip_norm)

    def _dygraph_clip(self, params_grads):
        out = []
        for p, g in params_grads:
            if g is None or not getattr(p, "need_clip", True):
                out.append((p, g))
                continue
            n = g._t.float().norm()
            scale = torch.clamp(self.clip_norm / torch.clamp(n, min=1e-30), max=1.0)
            g._t.mul_(scale.to(g._t.dtype))
            out.append((p, g))
        return out


class ClipGradByGlobalNorm(ClipGradBase):
    def __init__(self, clip_norm, group_name="default_group", auto_skip_clip=False):
        self.clip_norm = float(clip_norm)
        self.group_name = group_name
        self._mp_groups = []   # filled by fleet for hybrid parallel

    def global_norm_sq(self, grads, dist_grads=None):
        sq = _ops.global_norm_sq([g for g in grads])
        if dist_grads:
            dsq = _ops.global_norm_sq(dist_grads)
            for grp in self._mp_groups:
                import torch.distributed as dist
                dist.all_reduce(dsq, group=grp)
            sq = sq + dsq
        return sq

    def scale_factor(self, params_grads):
        """fp32 device scalar min(1, clip_norm / global_norm) over the clipped gradients, or None
        when no gradient takes part (the fused optimizers multiply it in as they read gradients)."""
        grads, dist_grads = self._split(params_grads)
        if not grads and not dist_grads:
            return None
        norm = torch.sqrt(self.global_norm_sq(grads, dist_grads))
        return torch.clamp(self.clip_norm / torch.clamp(norm, min=1e-6), max=1.0).float().reshape(1)

    def _split(self, params_grads):
        grads, dist_grads = [], []
        for p, g in params_grads:
            if g is None or not getattr(p, "need_clip", True):
                continue
            if getattr(p, "is_distributed", False) and self._mp_groups:
                dist_grads.append(g._t)
            else:
                grads.append(g._t)
        return grads, dist_grads

    def _dygraph_clip(self, params_grads):
        grads, dist_grads = self._split(params_grads)
        if not grads and not dist_grads:
            return params_grads
        sq = self.global_norm_sq(grads, dist_grads)
        norm = torch.sqrt(sq)
        scale = torch.clamp(self.clip_norm / torch.clamp(norm, min=1e-6), max=1.0)
        allg = grads + dist_grads
        by_dt = {}
        for g in allg:
            by_dt.setdefault(g.dtype, []).append(g)
        for dt, gs in by_dt.items():
            torch._foreach_mul_(gs, scale.to(dt))
        return params_grads


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False):
    params = [parameters] if isinstance(parameters, Tensor) else list(parameters)
    grads = [p._t.grad for p in params if p._t.grad is not None]
    if not grads:
        return _wrap(torch.tensor(0.0))
    total = torch.norm(torch.stack([torch.norm(g.float(), norm_type) for g in grads]), norm_type)
    if error_if_nonfinite and not torch.isfinite(total):
        raise RuntimeError("non-finite grad norm")
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in grads:
        g.mul_(coef.to(g.dtype))
    return _wrap(total)


def clip_grad_value_(parameters, clip_value):
    params = [parameters] if isinstance(parameters, Tensor) else list(parameters)
    for p in params:
        if p._t.grad is not None:
            p._t.grad.clamp_(-clip_value, clip_value)
