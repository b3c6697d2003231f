"""paddle.incubate.autotune.set_config (reference: python/paddle/incubate/autotune.py).

kernel.enable → let MIOpen/hipBLASLt benchmark algorithms (torch.backends.cudnn.benchmark);
layout.enable → prefer channels-last (NHWC) convolution layouts, the fast path on MI355X;
dataloader.enable → let the DataLoader tune its worker count on first use."""
from __future__ import annotations

import json
import warnings

import torch

__all__ = ["set_config", "get_config"]

_config = {"kernel": {"enable": False, "tuning_range": [1, 10]}, "layout": {"enable": False},
           "dataloader": {"enable": False, "tuning_steps": 500}}


def set_config(config=None):
    if config is None:
        config = {"kernel": {"enable": True}, "layout": {"enable": True}, "dataloader": {"enable": True}}
    if isinstance(config, str):
        with open(config) as f:
            config = json.load(f)
    for k, v in config.items():
        if k not in _config:
            warnings.warn(f"unknown autotune config key {k}")
            continue
        _config[k].update(v)
    torch.backends.cudnn.benchmark = bool(_config["kernel"]["enable"])
    from ..framework import flags
    flags.set_flags({"FLAGS_use_autotune": bool(_config["kernel"]["enable"]),
                     "FLAGS_conv_prefer_nhwc": bool(_config["layout"]["enable"])})


def get_config():
    return json.loads(json.dumps(_config))
