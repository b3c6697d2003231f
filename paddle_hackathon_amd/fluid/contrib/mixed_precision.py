"""``fluid.contrib.mixed_precision`` (reference: fluid/contrib/mixed_precision/decorator.py):
``decorate(optimizer, ...)`` -> an optimizer whose static ``minimize`` inserts the AMP
loss-scaling pass (static/passes.py insert_loss_scaling) and whose dygraph path uses GradScaler."""
from __future__ import annotations

from ...framework import core as _core

__all__ = ["decorate", "AutoMixedPrecisionLists", "CustomOpLists"]


class AutoMixedPrecisionLists:
    def __init__(self, custom_white_list=None, custom_black_list=None, custom_black_varnames=None):
        self.white_list = set(custom_white_list or [])
        self.black_list = set(custom_black_list or [])
        self.black_varnames = set(custom_black_varnames or [])


CustomOpLists = AutoMixedPrecisionLists


class _AMPOptimizer:
    def __init__(self, optimizer, amp_lists, init_loss_scaling, use_dynamic_loss_scaling, incr_every_n_steps,
                 decr_every_n_nan_or_inf, incr_ratio, decr_ratio, use_bf16):
        self._optimizer = optimizer
        self._lists = amp_lists
        self._cfg = dict(init_loss_scaling=init_loss_scaling, use_dynamic_loss_scaling=use_dynamic_loss_scaling,
                         incr_every_n_steps=incr_every_n_steps, decr_every_n_nan_or_inf=decr_every_n_nan_or_inf,
                         incr_ratio=incr_ratio, decr_ratio=decr_ratio)
        self._bf16 = use_bf16
        self._scaler = None

    def get_loss_scaling(self):
        """the current loss scale (a Variable-backed tensor after a static minimize)"""
        st = getattr(self, "_state", None)
        return st["scale"] if st is not None else self._cfg["init_loss_scaling"]

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        if not _core.in_dynamic_mode():
            from ...static.backward import append_backward, append_optimize_op
            from ...static import passes
            pg = append_backward(loss, parameter_list, no_grad_set)
            c = self._cfg
            pg, found, self._state = passes.insert_loss_scaling(
                loss.block.program, loss, pg, init_scale=c["init_loss_scaling"],
                incr_every_n_steps=c["incr_every_n_steps"], decr_every_n_nan_or_inf=c["decr_every_n_nan_or_inf"],
                incr_ratio=c["incr_ratio"], decr_ratio=c["decr_ratio"], dynamic=c["use_dynamic_loss_scaling"])
            return [append_optimize_op(self._optimizer, pg, found_inf=found)], pg
        from ...amp import GradScaler
        if self._scaler is None:
            c = self._cfg
            self._scaler = GradScaler(True, c["init_loss_scaling"], c["incr_ratio"], c["decr_ratio"],
                                      c["incr_every_n_steps"], c["decr_every_n_nan_or_inf"],
                                      c["use_dynamic_loss_scaling"])
        return self._scaler.minimize(self._optimizer, loss)

    def __getattr__(self, item):
        return getattr(self._optimizer, item)


def decorate(optimizer, amp_lists=None, init_loss_scaling=2 ** 15, incr_every_n_steps=1000,
             decr_every_n_nan_or_inf=2, incr_ratio=2.0, decr_ratio=0.8, use_dynamic_loss_scaling=True,
             use_pure_fp16=False, use_fp16_guard=None, use_bf16=False):
    return _AMPOptimizer(optimizer, amp_lists or AutoMixedPrecisionLists(), init_loss_scaling,
                         use_dynamic_loss_scaling, incr_every_n_steps, decr_every_n_nan_or_inf, incr_ratio,
                         decr_ratio, use_bf16)
