"""``fleet.metrics`` (reference: python/paddle/distributed/fleet/metrics/metric.py): metrics whose
statistics are summed (or max / min reduced) over all trainers before the final division — the
AUC from bucketed positive / negative counts, MAE / MSE / RMSE from error sums and instance
counts, accuracy from correct / total counts. Inputs are numpy arrays, Tensors or the names of
variables in ``scope``; one all-reduce per statistic over the default group (identity in a
single process)."""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.distributed as dist

__all__ = ["sum", "max", "min", "auc", "mae", "rmse", "mse", "acc"]

_builtin_sum, _builtin_max, _builtin_min = sum, max, min


def _value(x, scope=None):
    if isinstance(x, str):
        from ....static import global_scope
        s = scope or global_scope()
        v = s.find_var(x)
        x = v.get_tensor() if hasattr(v, "get_tensor") else v
    if hasattr(x, "_t"):
        x = x._t
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().double().numpy()
    return np.asarray(x, dtype=np.float64)


def _reduce(arr, op):
    a = np.array(arr, dtype=np.float64, copy=True)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.from_numpy(a)
        if dist.get_backend() == "nccl":
            t = t.cuda()
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        dist.all_reduce(t, op=rop)
        a = t.cpu().numpy()
    return a


def sum(input, scope=None, util=None):   # noqa: A001 (reference name)
    return _reduce(_value(input, scope), "sum")


def max(input, scope=None, util=None):   # noqa: A001
    return _reduce(_value(input, scope), "max")


def min(input, scope=None, util=None):   # noqa: A001
    return _reduce(_value(input, scope), "min")


def auc(stat_pos, stat_neg, scope=None, util=None):
    """global AUC from the bucketed positive / negative counts (the auc op's StatPos / StatNeg):
    trapezoids over the buckets from the highest threshold down"""
    pos = _reduce(_value(stat_pos, scope).reshape(-1), "sum")
    neg = _reduce(_value(stat_neg, scope).reshape(-1), "sum")
    area, tp, fp = 0.0, 0.0, 0.0
    for i in range(len(pos) - 1, -1, -1):
        ntp, nfp = tp + pos[i], fp + neg[i]
        area += (nfp - fp) * (tp + ntp) / 2.0
        tp, fp = ntp, nfp
    if tp <= 0 or fp <= 0:
        return 0.5
    return float(area / (tp * fp))


def mae(abserr, total_ins_num, scope=None, util=None):
    e = float(_reduce(_value(abserr, scope).reshape(-1), "sum")[0])
    n = float(_reduce(_value(total_ins_num, scope).reshape(-1), "sum")[0])
    return e / n if n else 0.0


def mse(sqrerr, total_ins_num, scope=None, util=None):
    e = float(_reduce(_value(sqrerr, scope).reshape(-1), "sum")[0])
    n = float(_reduce(_value(total_ins_num, scope).reshape(-1), "sum")[0])
    return e / n if n else 0.0


def rmse(sqrerr, total_ins_num, scope=None, util=None):
    return math.sqrt(mse(sqrerr, total_ins_num, scope, util))


def acc(correct, total, scope=None, util=None):
    c = float(_reduce(_value(correct, scope).reshape(-1), "sum")[0])
    t = float(_reduce(_value(total, scope).reshape(-1), "sum")[0])
    return c / t if t else 0.0
