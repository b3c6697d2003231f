"""``paddle.onnx.export`` (reference: python/paddle/onnx/export.py, which delegates to
paddle2onnx). Here the layer is traced through its torch compute graph on the CPU (so the
HIP kernels' portable fallbacks are what get exported) and written with torch's ONNX
exporter to ``{path}.onnx``."""
from __future__ import annotations

import os

import numpy as np
import torch

from .framework.core import Tensor, _wrap
from .framework import core as _core

__all__ = ["export"]


class _Adapter(torch.nn.Module):
    """Exposes the framework Layer's parameters as torch Parameters so the tracer emits them as
    ONNX initializers (their tensors are swapped in for the duration of the export)."""

    def __init__(self, layer):
        super().__init__()
        self.layer = layer
        self._saved = []
        for i, (n, p) in enumerate(layer.named_parameters()):
            tp = torch.nn.Parameter(p._t.detach(), requires_grad=False)
            self.register_parameter(f"p{i}", tp)
            self._saved.append((p, p._t))
            p._t = tp

    def restore(self):
        for p, t in self._saved:
            p._t = t

    def forward(self, *ts):
        out = self.layer(*[_wrap(t) for t in ts])
        if isinstance(out, (list, tuple)):
            return tuple(o._t for o in out)
        return out._t


def _allow_without_onnx_package():
    """torch serialises the ModelProto in C++; the python ``onnx`` package is only used to
    splice onnx-script functions into it, which our graphs never contain. When that package
    is absent (this image), make that splice a pass-through so export still works."""
    try:
        import onnx  # noqa: F401
        return
    except ImportError:
        pass
    from torch.onnx._internal.torchscript_exporter import onnx_proto_utils as u
    if not getattr(u._add_onnxscript_fn, "_pha_passthrough", False):
        def passthrough(model_bytes, custom_opsets):
            return model_bytes
        passthrough._pha_passthrough = True
        u._add_onnxscript_fn = passthrough


def export(layer, path, input_spec=None, opset_version=9, **configs):
    from .static import InputSpec
    if input_spec is None:
        raise ValueError("onnx.export needs input_spec")
    examples, names, dyn = [], [], {}
    for i, s in enumerate(input_spec):
        if isinstance(s, Tensor):
            examples.append(s._t.detach().cpu())
            names.append(s.name or f"x{i}")
            continue
        shape = [d if d is not None and d >= 0 else 1 for d in s.shape]
        dt = _core.convert_dtype(s.dtype) or torch.float32
        examples.append(torch.zeros(shape, dtype=dt) if dt.is_floating_point else torch.zeros(shape, dtype=dt))
        names.append(s.name or f"x{i}")
        axes = {k: f"d{i}_{k}" for k, d in enumerate(s.shape) if d is None or d < 0}
        if axes:
            dyn[names[-1]] = axes
    was_training = layer.training
    layer.eval()
    prev = _core._default_device
    _core._default_device = torch.device("cpu")
    try:
        out_path = path if path.endswith(".onnx") else path + ".onnx"
        d = os.path.dirname(out_path)
        if d:
            os.makedirs(d, exist_ok=True)
        ad = _Adapter(layer)
        try:
            _allow_without_onnx_package()
            with torch.no_grad():
                torch.onnx.export(ad, tuple(examples), out_path, input_names=names,
                                  opset_version=max(opset_version, 9), dynamic_axes=dyn or None, dynamo=False)
        finally:
            ad.restore()
    finally:
        _core._default_device = prev
        if was_training:
            layer.train()
    return out_path
