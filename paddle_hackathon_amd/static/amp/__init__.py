"""``paddle.static.amp`` (reference: python/paddle/fluid/contrib/mixed_precision/{decorator,
fp16_utils,fp16_lists}.py and bf16/, re-exported as paddle.static.amp).

* ``decorate(optimizer, ...)``: an optimizer whose static ``minimize`` first rewrites the forward
  (the white-listed compute ops — matmul / linear / conv2d / bmm / einsum / mm and the custom white
  list — run in fp16, static/passes.py ``cast_forward_to``; with ``use_fp16_guard`` only the ops
  recorded under ``fp16_guard()``), then builds the backward and the dynamic loss scaling
  (check_finite_and_unscale / update_loss_scaling, the optimizer skipping overflow steps);
* ``cast_model_to_fp16`` / ``cast_parameters_to_fp16``: pure fp16 programs (parameters stored in
  fp16, every op computing in it);
* ``bf16``: the same for bfloat16 (no loss scaling needed)."""
from __future__ import annotations

import contextlib

import torch

from ...fluid.contrib.mixed_precision import AutoMixedPrecisionLists, CustomOpLists, _AMPOptimizer  # noqa: F401
from .. import passes as _passes
from ..program import default_main_program

__all__ = ["decorate", "CustomOpLists", "AutoMixedPrecisionLists", "fp16_guard", "cast_model_to_fp16",
           "cast_parameters_to_fp16", "bf16"]

_WHITE = ("matmul", "linear", "conv2d", "bmm", "einsum", "mm", "conv2d_transpose", "conv1d", "conv3d")
_GUARD = [False]


@contextlib.contextmanager
def fp16_guard():
    """ops recorded inside run in fp16 when the decorator has ``use_fp16_guard=True``"""
    prog = default_main_program()
    blk = prog.current_block()
    start = len(blk.ops)
    _GUARD[0] = True
    try:
        yield
    finally:
        _GUARD[0] = False
        for op in blk.ops[start:]:
            op.attrs["fp16_guard"] = True


def _white(amp_lists):
    names = set(_WHITE)
    if amp_lists is not None:
        names |= set(getattr(amp_lists, "white_list", ()))
        names -= set(getattr(amp_lists, "black_list", ()))
    return tuple(names)


def _cast(prog, dtype, amp_lists=None, guard=False, everything=False):
    ops = prog.global_block().ops
    if guard:   # only the guarded ops
        keep = [op for op in ops if not op.attrs.get("fp16_guard")]
        for op in keep:
            op.attrs["amp_cast"] = "skip"
        _passes.cast_forward_to(prog, dtype, white=_white(amp_lists) if not everything else
                                tuple({op.type.rsplit(".", 1)[-1] for op in ops}))
        for op in keep:
            if op.attrs.get("amp_cast") == "skip":
                del op.attrs["amp_cast"]
        return prog
    white = tuple({op.type.rsplit(".", 1)[-1] for op in ops}) if everything else _white(amp_lists)
    return _passes.cast_forward_to(prog, dtype, white=white)


class _StaticAMP(_AMPOptimizer):
    def __init__(self, *a, dtype=torch.float16, use_fp16_guard=False, pure=False, **kw):
        super().__init__(*a, **kw)
        self._dtype, self._guard, self._pure = dtype, bool(use_fp16_guard), pure

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        from ...framework import core as _core
        if not _core.in_dynamic_mode():
            _cast(loss.block.program, self._dtype, self._lists, self._guard, everything=self._pure)
        return super().minimize(loss, startup_program, parameter_list, no_grad_set)

    def amp_init(self, place=None, scope=None, test_program=None, use_fp16_test=False):
        """pure fp16: cast the initialised parameters (reference: OptimizerWithMixedPrecision.amp_init)"""
        if self._pure:
            cast_parameters_to_fp16(place, default_main_program(), scope)


def decorate(optimizer, amp_lists=None, init_loss_scaling=2 ** 15, incr_every_n_steps=1000,
             decr_every_n_nan_or_inf=2, incr_ratio=2.0, decr_ratio=0.8, use_dynamic_loss_scaling=True,
             use_pure_fp16=False, use_fp16_guard=None):
    return _StaticAMP(optimizer, amp_lists or AutoMixedPrecisionLists(), init_loss_scaling, use_dynamic_loss_scaling,
                      incr_every_n_steps, decr_every_n_nan_or_inf, incr_ratio, decr_ratio, False,
                      dtype=torch.float16, use_fp16_guard=bool(use_fp16_guard) if use_fp16_guard is not None
                      else use_pure_fp16, pure=use_pure_fp16)


def cast_model_to_fp16(program, amp_lists=None, use_fp16_guard=True, dtype=torch.float16):
    """every forward op of ``program`` (the guarded ones with ``use_fp16_guard``) computes in fp16"""
    return _cast(program, dtype, amp_lists, use_fp16_guard, everything=True)


def cast_parameters_to_fp16(place=None, program=None, scope=None, to_fp16_var_names=None, dtype=torch.float16):
    """the program's floating-point parameters stored in fp16 (in place)"""
    program = program or default_main_program()
    names = set(to_fp16_var_names) if to_fp16_var_names else None
    for p in program.all_parameters():
        if p._t.is_floating_point() and (names is None or p.name in names):
            with torch.no_grad():
                p._t = p._t.to(dtype)


from . import bf16  # noqa: E402,F401
