"""Automatic mixed precision (reference: python/paddle/amp/{auto_cast,grad_scaler}.py,
python/paddle/fluid/dygraph/amp/*, operators/amp/{check_finite_and_unscale,update_loss_scaling}_op.cu).

O1: per-op casting through PyTorch-ROCm autocast (GEMM/conv white list → bf16/fp16
on MFMA, reductions/norm/softmax black list → fp32).
O2: ``decorate`` casts the model's parameters to the low-precision dtype (norm
layers stay fp32) and the optimizer keeps fp32 master weights (multi_precision).
"""
from __future__ import annotations

import contextlib

import torch

from ..framework.core import Tensor, _wrap, convert_dtype, default_device
from .. import ops as _ops

__all__ = ["auto_cast", "GradScaler", "decorate", "AmpScaler", "amp_guard", "is_float16_supported", "is_bfloat16_supported"]

_amp_state = {"level": "O0", "dtype": torch.float16, "enabled": False}


def amp_state():
    return _amp_state


@contextlib.contextmanager
def auto_cast(enable=True, custom_white_list=None, custom_black_list=None, level="O1", dtype="float16"):
    dt = convert_dtype(dtype)
    prev = dict(_amp_state)
    if not enable or level == "O0":
        yield
        return
    _amp_state.update(level=level, dtype=dt, enabled=True)
    dev = default_device().type
    try:
        if level == "O2":
            # parameters already cast by decorate(); keep autocast for mixed inputs
            with torch.autocast(device_type=dev, dtype=dt):
                yield
        else:
            with torch.autocast(device_type=dev, dtype=dt):
                yield
    finally:
        _amp_state.clear()
        _amp_state.update(prev)


amp_guard = auto_cast


def is_float16_supported(device=None):
    return True


def is_bfloat16_supported(device=None):
    return True


_KEEP_FP32 = ("BatchNorm", "LayerNorm", "GroupNorm", "InstanceNorm", "SyncBatchNorm", "RMSNorm")


def decorate(models, optimizers=None, level="O1", dtype="float16", master_weight=None, save_dtype=None,
             excluded_layers=None):
    if level == "O1":
        return (models, optimizers) if optimizers is not None else models
    dt = convert_dtype(dtype)
    mlist = models if isinstance(models, (list, tuple)) else [models]
    excluded = tuple(excluded_layers) if excluded_layers else ()
    for m in mlist:
        for layer in m.sublayers(include_self=True):
            name = type(layer).__name__
            if any(k in name for k in _KEEP_FP32) or (excluded and isinstance(layer, excluded)):
                continue
            for p in layer._parameters.values():
                if p is not None and p._t.is_floating_point():
                    rg = p._t.requires_grad
                    p._t = p._t.detach().to(dt).requires_grad_(rg)
        m._casted_by_pure_fp16 = True
        m._amp_save_dtype = save_dtype
    if optimizers is not None:
        olist = optimizers if isinstance(optimizers, (list, tuple)) else [optimizers]
        for o in olist:
            o._multi_precision = True if master_weight is None else bool(master_weight)
        return models, optimizers
    return models


class GradScaler:
    """Dynamic loss scaling (reference: python/paddle/amp/grad_scaler.py)."""

    def __init__(self, enable=True, init_loss_scaling=2.0 ** 15, incr_ratio=2.0, decr_ratio=0.5,
                 incr_every_n_steps=1000, decr_every_n_nan_or_inf=2, use_dynamic_loss_scaling=True):
        self._enable = enable
        self._scale = float(init_loss_scaling)
        self._incr_ratio, self._decr_ratio = incr_ratio, decr_ratio
        self._incr_every_n_steps, self._decr_every_n_nan_or_inf = incr_every_n_steps, decr_every_n_nan_or_inf
        self._use_dynamic = use_dynamic_loss_scaling
        self._good_steps = 0
        self._bad_steps = 0
        self._found_inf = False
        self._unscaled = False

    def is_enable(self):
        return self._enable

    def is_use_dynamic_loss_scaling(self):
        return self._use_dynamic

    def get_init_loss_scaling(self):
        return self._scale

    def set_init_loss_scaling(self, v):
        self._scale = float(v)

    def scale(self, var):
        if not self._enable:
            return var
        return _wrap(var._t * self._scale)

    def _grads(self, optimizer):
        return [p._t.grad for p in optimizer._parameter_list or [] if p._t.grad is not None]

    def unscale_(self, optimizer):
        if not self._enable or self._unscaled:
            return
        grads = self._grads(optimizer)
        found = _ops.check_finite_and_unscale_(grads, 1.0 / self._scale)
        self._found_inf = bool(found)
        self._unscaled = True

    def minimize(self, optimizer, *args, **kwargs):
        self.step(optimizer)
        self.update()
        return None, None

    def step(self, optimizer):
        if not self._enable:
            optimizer.step()
            return
        self.unscale_(optimizer)
        if not self._found_inf:
            optimizer.step()

    def update(self):
        if not self._enable:
            return
        if self._use_dynamic:
            if self._found_inf:
                self._good_steps = 0
                self._bad_steps += 1
                if self._bad_steps == self._decr_every_n_nan_or_inf:
                    self._scale = max(self._scale * self._decr_ratio, 1.0)
                    self._bad_steps = 0
            else:
                self._bad_steps = 0
                self._good_steps += 1
                if self._good_steps == self._incr_every_n_steps:
                    self._scale *= self._incr_ratio
                    self._good_steps = 0
        self._unscaled = False
        self._found_inf = False

    def state_dict(self):
        return {"scale": self._scale, "incr_ratio": self._incr_ratio, "decr_ratio": self._decr_ratio,
                "incr_every_n_steps": self._incr_every_n_steps, "decr_every_n_nan_or_inf": self._decr_every_n_nan_or_inf,
                "incr_count": self._good_steps, "decr_count": self._bad_steps,
                "use_dynamic_loss_scaling": self._use_dynamic}

    def load_state_dict(self, sd):
        self._scale = float(sd["scale"])
        self._good_steps = sd.get("incr_count", 0)
        self._bad_steps = sd.get("decr_count", 0)

    set_state_dict = load_state_dict


AmpScaler = GradScaler
