"""``save_dygraph`` / ``load_dygraph`` (reference: python/paddle/fluid/dygraph/checkpoint.py):
``{path}.pdparams`` for a Layer's state dict, ``{path}.pdopt`` for an optimizer's."""
from __future__ import annotations

import os

from ...framework.io import save as _save, load as _load

__all__ = ["save_dygraph", "load_dygraph"]


def save_dygraph(state_dict, model_path):
    is_opt = any(k in state_dict for k in ("LR_Scheduler", "master_weights")) or \
        any("_moment" in k or "velocity" in k or "beta1_pow" in k for k in state_dict)
    suffix = ".pdopt" if is_opt else ".pdparams"
    d = os.path.dirname(model_path)
    if d:
        os.makedirs(d, exist_ok=True)
    _save(state_dict, model_path + suffix)


def load_dygraph(model_path, **configs):
    """-> (param_dict, optimizer_dict); either is None when its file is absent"""
    base = model_path
    for s in (".pdparams", ".pdopt"):
        if base.endswith(s):
            base = base[:-len(s)]
    params = _load(base + ".pdparams", return_numpy=True) if os.path.exists(base + ".pdparams") else None
    opt = _load(base + ".pdopt", return_numpy=True) if os.path.exists(base + ".pdopt") else None
    return params, opt
