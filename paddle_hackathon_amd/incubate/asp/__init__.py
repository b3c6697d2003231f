"""Automatic SParsity — n:m structured pruning (reference: python/paddle/fluid/contrib/
sparsity/{asp,utils}.py, exported as paddle.incubate.asp).

Masks are n:m along the GEMM reduction dimension (K): for a Linear weight [in, out] the
groups of ``m`` run along ``in``; for a conv weight [out, in, kh, kw] along ``in``. 2:4 along
K is exactly the operand layout CDNA4's sparse MFMA (``v_smfmac``) consumes, so a pruned
model can later be lowered onto sparse matrix cores without re-pruning."""
from __future__ import annotations

import enum
import itertools

import numpy as np
import torch

from ...framework.core import Tensor, _wrap

__all__ = ["calculate_density", "decorate", "prune_model", "set_excluded_layers", "reset_excluded_layers",
           "MaskAlgo", "CheckMethod", "create_mask", "check_sparsity", "add_supported_layer"]


class MaskAlgo(enum.Enum):
    MASK_1D = "get_mask_1d"
    MASK_2D_GREEDY = "get_mask_2d_greedy"
    MASK_2D_BEST = "get_mask_2d_best"


class CheckMethod(enum.Enum):
    CHECK_1D = "check_mask_1d"
    CHECK_2D = "check_mask_2d"

    @staticmethod
    def get_checking_method(mask_algo):
        return CheckMethod.CHECK_1D if mask_algo == MaskAlgo.MASK_1D else CheckMethod.CHECK_2D


def calculate_density(x):
    a = x.numpy() if isinstance(x, Tensor) else np.asarray(x)
    a = a.reshape(-1)
    return float(np.count_nonzero(a)) / a.size


def _pad_cols(mat, m):
    r = mat.shape[1] % m
    if r:
        mat = torch.cat([mat, mat.new_zeros(mat.shape[0], m - r)], 1)
    return mat


def get_mask_1d(mat, n, m):
    """Keep the n largest-|w| of every m consecutive entries in each row."""
    t = torch.as_tensor(mat, dtype=torch.float64)
    rows, cols = t.shape
    p = _pad_cols(t, m).reshape(-1, m).abs()
    idx = torch.argsort(p, dim=1)[:, : m - n]  # smallest m-n are zeroed
    mask = torch.ones_like(p)
    mask.scatter_(1, idx, 0.0)
    return mask.reshape(rows, -1)[:, :cols].numpy()


def check_mask_1d(mat, n, m):
    t = torch.as_tensor(np.asarray(mat), dtype=torch.float64)
    if t.dim() == 1:
        t = t.reshape(1, -1)
    p = _pad_cols(t, m).reshape(-1, m)
    return bool(((p != 0).sum(1) <= n).all())


def _blocks_2d(t, m):
    rows, cols = t.shape
    pr = (m - rows % m) % m
    pc = (m - cols % m) % m
    p = torch.nn.functional.pad(t, (0, pc, 0, pr))
    R, C = p.shape
    return p.reshape(R // m, m, C // m, m).permute(0, 2, 1, 3).reshape(-1, m, m), (R, C)


def _unblock_2d(b, shape, m, rows, cols):
    R, C = shape
    return b.reshape(R // m, C // m, m, m).permute(0, 2, 1, 3).reshape(R, C)[:rows, :cols]


def check_mask_2d(mat, n, m):
    t = torch.as_tensor(np.asarray(mat), dtype=torch.float64)
    if t.dim() == 1:
        t = t.reshape(1, -1)
    b, _ = _blocks_2d(t, m)
    nz = b != 0
    return bool((nz.sum(1) <= n).all() and (nz.sum(2) <= n).all())


def get_mask_2d_greedy(mat, n, m):
    """Per m×m block, greedily keep the largest entries while every row and column keeps ≤ n."""
    t = torch.as_tensor(mat, dtype=torch.float64)
    rows, cols = t.shape
    b, shape = _blocks_2d(t.abs(), m)
    out = torch.zeros_like(b)
    for k in range(b.shape[0]):
        blk = b[k]
        order = torch.argsort(blk.reshape(-1), descending=True)
        rc, cc = [0] * m, [0] * m
        for o in order.tolist():
            r, c = divmod(o, m)
            if rc[r] < n and cc[c] < n:
                out[k, r, c] = 1
                rc[r] += 1
                cc[c] += 1
    return _unblock_2d(out, shape, m, rows, cols).numpy()


_PATTERNS = {}


def _valid_2d_patterns(n, m):
    key = (n, m)
    if key not in _PATTERNS:
        rowsel = [r for r in itertools.product([0, 1], repeat=m) if sum(r) == n]
        pats = []
        for combo in itertools.product(rowsel, repeat=m):
            a = np.asarray(combo)
            if (a.sum(0) == n).all():
                pats.append(a)
        _PATTERNS[key] = torch.as_tensor(np.stack(pats), dtype=torch.float64)
    return _PATTERNS[key]


def get_mask_2d_best(mat, n, m):
    """Per m×m block, the valid n:m (rows and columns) pattern maximising kept |w|."""
    t = torch.as_tensor(mat, dtype=torch.float64)
    rows, cols = t.shape
    b, shape = _blocks_2d(t.abs(), m)
    pats = _valid_2d_patterns(n, m)  # [P, m, m]
    score = torch.einsum("kij,pij->kp", b, pats)
    best = pats[score.argmax(1)]
    return _unblock_2d(best, shape, m, rows, cols).numpy()


_FUNCS = {"get_mask_1d": get_mask_1d, "get_mask_2d_greedy": get_mask_2d_greedy,
          "get_mask_2d_best": get_mask_2d_best, "check_mask_1d": check_mask_1d, "check_mask_2d": check_mask_2d}


def create_mask(tensor, func_name=MaskAlgo.MASK_1D, n=2, m=4):
    a = tensor.numpy() if isinstance(tensor, Tensor) else np.asarray(tensor)
    shape, dtype = a.shape, a.dtype
    f = _FUNCS[func_name.value]
    t = a.astype(np.float64)
    if len(shape) == 1:
        t = t.reshape(1, shape[0])
    elif len(shape) == 3:
        t = t.reshape(shape[0] * shape[1], shape[2])
    elif len(shape) == 4:  # (h, w, in, out) -> (h*w*out, in)
        t = t.transpose(0, 1, 3, 2).reshape(shape[0] * shape[1] * shape[3], shape[2])
        mask = f(t, n=n, m=m)
        return mask.reshape(shape[0], shape[1], shape[3], shape[2]).transpose(0, 1, 3, 2).astype(dtype)
    elif len(shape) != 2:
        raise ValueError(f"create_mask supports dims <= 4, got {len(shape)}")
    return f(t, n=n, m=m).reshape(shape).astype(dtype)


def check_sparsity(tensor, func_name=CheckMethod.CHECK_1D, n=2, m=4):
    a = tensor.numpy() if isinstance(tensor, Tensor) else np.asarray(tensor)
    shape = a.shape
    t = a.astype(np.float64)
    if len(shape) == 1:
        t = t.reshape(1, shape[0])
    elif len(shape) == 3:
        t = t.reshape(shape[0] * shape[1], shape[2])
    elif len(shape) == 4:
        t = t.transpose(0, 1, 3, 2).reshape(shape[0] * shape[1] * shape[3], shape[2])
    return _FUNCS[func_name.value](t, n=n, m=m)


# --------------------------------------------------------------------------- model-level API
_excluded = set()
_supported = {"Linear", "Conv2D", "Conv1D", "Conv3D", "FusedLinear"}
_masks = {}  # param name -> torch mask (device, param dtype)


def add_supported_layer(layer, pruning_func=None):
    _supported.add(layer if isinstance(layer, str) else layer.__name__)


def set_excluded_layers(param_names=None, main_program=None):
    if isinstance(param_names, str):
        param_names = [param_names]
    _excluded.update(param_names or [])


def reset_excluded_layers(main_program=None):
    _excluded.clear()


def _prunable(model):
    for lname, layer in model.named_sublayers(include_self=True):
        if type(layer).__name__ not in _supported:
            continue
        w = getattr(layer, "weight", None)
        if w is None or w.ndim < 2:
            continue
        if w.name in _excluded or lname in _excluded or any(e and e in w.name for e in _excluded):
            continue
        yield layer, w


def _weight_mask(layer, w, n, m, algo):
    a = w._t.detach().float().cpu().numpy()
    name = type(layer).__name__
    if name in ("Linear", "FusedLinear") and a.ndim == 2:
        # weight [in, out]: groups run along `in` (K of the GEMM)
        return create_mask(a.T, algo, n, m).T
    if a.ndim == 4:  # conv [out, in, kh, kw] -> (kh, kw, in, out) layout of create_mask
        t = a.transpose(2, 3, 1, 0)
        return create_mask(t, algo, n, m).transpose(3, 2, 0, 1)
    return create_mask(a, algo, n, m)


def prune_model(model, n=2, m=4, mask_algo="mask_1d", with_mask=True):
    algo = mask_algo if isinstance(mask_algo, MaskAlgo) else MaskAlgo["MASK_" + mask_algo[len("mask_"):].upper()]
    masks = {}
    with torch.no_grad():
        for layer, w in _prunable(model):
            mk = torch.as_tensor(np.ascontiguousarray(_weight_mask(layer, w, n, m, algo)), device=w._t.device,
                                 dtype=w._t.dtype)
            w._t.mul_(mk)
            masks[w.name] = mk
            if with_mask:
                _masks[w.name] = mk
    return {k: _wrap(v) for k, v in masks.items()}


class OptimizerWithSparsityGuarantee:
    """Wraps an optimizer: after every step the n:m masks are re-applied so pruned weights stay 0."""

    def __init__(self, optimizer):
        self._optimizer = optimizer

    def __getattr__(self, item):
        return getattr(self._optimizer, item)

    @torch.no_grad()
    def _apply_masks(self):
        for p in self._optimizer._parameter_list or []:
            mk = _masks.get(p.name)
            if mk is not None:
                p._t.mul_(mk)
                mw = self._optimizer._master_weights.get(p.name) if hasattr(self._optimizer, "_master_weights") else None
                if mw is not None:
                    mw._t.mul_(mk.to(mw._t.dtype))

    def step(self):
        self._optimizer.step()
        self._apply_masks()

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        out = self._optimizer.minimize(loss, startup_program, parameters, no_grad_set)
        self._apply_masks()
        return out

    def state_dict(self):
        return self._optimizer.state_dict()

    def set_state_dict(self, sd):
        return self._optimizer.set_state_dict(sd)


def decorate(optimizer):
    return OptimizerWithSparsityGuarantee(optimizer)
