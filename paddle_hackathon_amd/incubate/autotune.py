"""paddle.incubate.autotune.set_config (reference: python/paddle/incubate/autotune.py).

kernel.enable → time the own conv kernels' tile candidates for shapes missing from the in-tree
table (ops/conv_gemm.py) and let MIOpen benchmark algorithms (torch.backends.cudnn.benchmark);
layout.enable → prefer channels-last (NHWC) convolution layouts, the fast path on MI355X;
dataloader.enable → let the DataLoader tune its worker count on first use.

GEMM algorithm selection (the reference's kernel autotune for matmul, phi/kernels/autotune/)
maps onto PyTorch's TunableOp over hipBLASLt/rocBLAS solutions: ``enable_gemm_tuning(tune=True)``
benchmarks every solution for each new GEMM shape and writes the winners to a CSV;
``enable_gemm_tuning()`` (tune=False) only loads the in-tree database
(``paddle_hackathon_amd/tuning/gemm_tunableop_gfx950.csv``) so a run pays no tuning cost."""
from __future__ import annotations

import json
import os
import warnings

import torch

__all__ = ["set_config", "get_config", "enable_gemm_tuning", "GEMM_TUNING_DB"]

GEMM_TUNING_DB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning",
                              "gemm_tunableop_gfx950.csv")


def enable_gemm_tuning(tune=False, filename=None, max_tuning_ms=30):
    """Turn on TunableOp GEMM dispatch. Returns the number of tuned entries loaded (or -1
    when tuning writes to ``filename`` at process exit)."""
    import torch.cuda.tunable as tun
    path = filename or GEMM_TUNING_DB
    tun.enable(True)
    if tune:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        tun.set_filename(path, False)
        tun.set_max_tuning_duration(int(max_tuning_ms))
        tun.tuning_enable(True)
        return -1
    tun.tuning_enable(False)
    if not os.path.exists(path):
        tun.enable(False)
        return 0
    ok = tun.read_file(path)
    if not ok:
        warnings.warn(f"GEMM tuning database {path} rejected (library versions changed?)")
        tun.enable(False)
        return 0
    return sum(1 for line in open(path) if line and not line.startswith("Validator"))

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
    from ..ops import conv_gemm
    conv_gemm.set_timing_autotune(_config["kernel"]["enable"])
    from ..framework import flags
    flags.set_flags({"FLAGS_use_autotune": bool(_config["kernel"]["enable"]),
                     "FLAGS_conv_prefer_nhwc": bool(_config["layout"]["enable"])})


def get_config():
    return json.loads(json.dumps(_config))
