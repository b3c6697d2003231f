"""Hot-path ops on torch tensors, backed by our gfx950 HIP kernel library.

Every function here takes/returns ``torch.Tensor``. On a HIP device with a
supported dtype the work goes to ``libpha_kernels.so`` (csrc/kernels/*.hip,
built for ``--offload-arch=gfx950``, called through a C ABI on the current
HIP stream); on CPU the PyTorch reference path runs (that path is also what
the numerics tests compare the HIP kernels against).

If a GPU is visible and the library is missing, import raises — GPU runs must
never silently fall back to the reference path (set ``PHA_ALLOW_FALLBACK=1``
to override for debugging).
"""
from __future__ import annotations

from ._lib import native_available, lib, require_native  # noqa: F401
from .fused import (  # noqa: F401
    gelu, bias_gelu, softmax, layer_norm, rms_norm, softmax_cross_entropy, embedding,
    fused_adam_, fused_momentum_, flash_attention, flash_attention_qkvpacked, bias_dropout_residual_layer_norm,
    global_norm_sq, scale_grads_, check_finite_and_unscale_, batch_norm_train, add_relu,
)
