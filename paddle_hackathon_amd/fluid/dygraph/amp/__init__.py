"""``fluid.dygraph.amp`` (reference: python/paddle/fluid/dygraph/amp/{auto_cast,loss_scaler}.py)."""
from __future__ import annotations

from ....amp import auto_cast, decorate, GradScaler

__all__ = ["amp_guard", "amp_decorate", "AmpScaler", "OptimizerState"]


def amp_guard(enable=True, custom_white_list=None, custom_black_list=None, level="O1", dtype="float16"):
    return auto_cast(enable, custom_white_list, custom_black_list, level, dtype)


def amp_decorate(models, optimizers=None, level="O1", master_weight=None, save_dtype=None):
    return decorate(models, optimizers, level, master_weight=master_weight, save_dtype=save_dtype)


class OptimizerState:
    INIT, UNSCALED, STEPPED = 0, 1, 2


class AmpScaler(GradScaler):
    def __init__(self, enable=True, init_loss_scaling=2. ** 15, incr_ratio=2.0, decr_ratio=0.5,
                 incr_every_n_steps=1000, decr_every_n_nan_or_inf=1, use_dynamic_loss_scaling=True):
        super().__init__(enable, init_loss_scaling, incr_ratio, decr_ratio, incr_every_n_steps,
                         decr_every_n_nan_or_inf, use_dynamic_loss_scaling)

    def minimize(self, optimizer, *args, **kwargs):
        r = super().minimize(optimizer, *args, **kwargs)
        after = getattr(optimizer, "_fluid_after_step", None)
        if after is not None:
            after()
        return r
