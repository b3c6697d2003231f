"""Gradient clipping (reference: python/paddle/fluid/clip.py).

``ClipGradByGlobalNorm`` computes the global norm with one multi-tensor HIP
reduction (ops.global_norm_sq) and scales all grads in place; under tensor /
pipeline / sharding parallelism the squared norm is all-reduced across the hybrid
"check" group first (see the class), matching HybridParallelClipGrad.
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
    """Global-norm clip. Under hybrid parallelism fleet sets ``_check_group`` (every rank that
    shares this rank's data-parallel coordinate: the mp x pp x sharding ranks) and ``_mp_degree``.
    The squared norm is then reduced with ONE all-reduce over that group (reference
    ``hybrid_parallel_optimizer.py:122-139`` issues up to three):

      * tensor-parallel-split gradients (``p.is_distributed``) are disjoint slices: summed;
      * replicated gradients are identical on the mp ranks of one pipeline stage: summed over the
        group and divided by the mp degree, which leaves the sum over pipeline stages and
        sharding owners;
      * a weight shared by pipeline stages (the tied embedding; ``is_firstly_shared`` False on
        every stage but the first that holds it) is counted once, but still scaled everywhere.

    The collective is issued even when this rank has no clipped gradient, so ranks never
    disagree on the number of collectives."""

    def __init__(self, clip_norm, group_name="default_group", auto_skip_clip=False):
        self.clip_norm = float(clip_norm)
        self.group_name = group_name
        self._check_group = None   # torch ProcessGroup, set by fleet for hybrid parallel
        self._mp_degree = 1

    def _split(self, params_grads):
        """-> (clipped grads, replicated grads counted in the norm, distributed grads counted)."""
        scaled, rep, dist_g = [], [], []
        for p, g in params_grads:
            if g is None or not getattr(p, "need_clip", True):
                continue
            scaled.append(g._t)
            if getattr(p, "is_firstly_shared", True) is False:
                continue
            (dist_g if getattr(p, "is_distributed", False) else rep).append(g._t)
        return scaled, rep, dist_g

    def global_norm_sq(self, rep, dist_g, device=None):
        dev = (rep or dist_g)[0].device if (rep or dist_g) else device
        sq = _ops.global_norm_sq(rep) if rep else torch.zeros((), dtype=torch.float32, device=dev)
        if self._check_group is not None:
            import torch.distributed as dist
            sq = sq.reshape(1).float()
            if self._mp_degree > 1:
                sq = sq / float(self._mp_degree)
            if dist_g:
                sq = sq + _ops.global_norm_sq(dist_g).float()
            if sq.device.type == "cpu" and dist.get_backend(self._check_group) == "nccl":
                # host-side gradients (sharding offload): RCCL needs a device tensor
                dev = torch.device("cuda", torch.cuda.current_device())
                red = sq.to(dev)
                dist.all_reduce(red, group=self._check_group)
                return red.to(sq.device).reshape(())
            dist.all_reduce(sq, group=self._check_group)
            return sq.reshape(())
        if dist_g:
            sq = sq + _ops.global_norm_sq(dist_g)
        return sq

    def _device_of(self, params_grads):
        for p, _ in params_grads:
            return p._t.device
        if getattr(self, "_device", None) is not None:
            return self._device
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")

    def scale_factor(self, params_grads):
        """fp32 device scalar min(1, clip_norm / global_norm) over the clipped gradients, or None
        when no gradient takes part and no group needs the collective (the fused optimizers
        multiply it in as they read gradients)."""
        scaled, rep, dist_g = self._split(params_grads)
        if not scaled and self._check_group is None:
            return None
        norm = torch.sqrt(self.global_norm_sq(rep, dist_g, self._device_of(params_grads)))
        return torch.clamp(self.clip_norm / torch.clamp(norm, min=1e-6), max=1.0).float().reshape(1)

    def _dygraph_clip(self, params_grads):
        scaled, rep, dist_g = self._split(params_grads)
        if not scaled and self._check_group is None:
            return params_grads
        norm = torch.sqrt(self.global_norm_sq(rep, dist_g, self._device_of(params_grads)))
        scale = torch.clamp(self.clip_norm / torch.clamp(norm, min=1e-6), max=1.0)
        by_dt = {}
        for g in scaled:
            by_dt.setdefault(g.dtype, []).append(g)
        for dt, gs in by_dt.items():
            torch._foreach_mul_(gs, scale.to(device=gs[0].device, dtype=dt))
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
