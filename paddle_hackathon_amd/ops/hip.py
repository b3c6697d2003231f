"""ctypes bindings to ``libpha_kernels.so`` (torch tensors in, torch tensors out).

Each call passes raw device pointers and the *current* torch HIP stream, so the
kernels order correctly with PyTorch-ROCm's own work and are capturable in HIP
graphs. Shape preconditions are checked here on the host before any launch
(a kernel reading out of bounds can take the whole GPU node down).
"""
from __future__ import annotations

import ctypes
from ctypes import c_uint, c_int, c_long, c_float, c_void_p

import numpy as np
import torch

from . import _lib

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
_sigs_done = False


def _L():
    global _sigs_done
    L = _lib.lib
    if L is None:
        raise RuntimeError("libpha_kernels.so not loaded")
    if not _sigs_done:
        P, I, F, LG = c_void_p, c_int, c_float, c_long
        sig = {
            "pha_layer_norm_fwd": [I, I, P, P, P, P, P, P, I, I, F, P],
            "pha_layer_norm_bwd": [I, I, P, P, P, P, P, P, P, P, P, P, I, I, I, P],
            "pha_layer_norm_bwd_nblocks": [I, I],
            "pha_layer_norm_fwd2": [I, I, P, P, P, P, P, P, P, P, I, I, F, P],
            "pha_layer_norm_bwd2": [I, I, P, P, P, P, P, P, P, P, P, P, P, I, I, I, P],
            "pha_layer_norm_bwd3": [I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, P],
            "pha_bdrln_fwd2": [I, I, I, P, P, P, P, P, P, P, P, P, I, I, F, c_uint, c_uint, F, P, P],
            "pha_col_sum_rows": [I, P, P, I, I, P],
            "pha_bdrln_fwd": [I, I, P, P, P, P, P, P, P, P, P, I, I, F, c_uint, c_uint, F, P],
            "pha_dropout_bias_bwd": [I, I, P, P, P, P, I, I, I, c_uint, c_uint, F, P, P],
            "pha_layer_norm_dropout_bwd": [I, I, P, P, P, P, P, P, P, P, P, P, P, I, I, I, c_uint, c_uint, F, P, P],
            "pha_softmax_fwd": [I, P, P, I, I, P],
            "pha_softmax_bwd": [I, P, P, P, I, I, P],
            "pha_softmax_ce_fwd": [I, P, P, P, P, LG, I, I, P],
            "pha_softmax_ce_bwd": [I, P, P, P, P, P, LG, I, I, P],
            "pha_bias_gelu_fwd": [I, P, P, P, LG, I, I, P],
            "pha_bias_gelu_bwd": [I, P, P, P, P, LG, I, I, P],
            "pha_embedding_fwd": [P, P, P, LG, I, LG, P],
            "pha_embedding_bwd": [I, P, P, P, LG, I, LG, LG, P, I, P],
            "pha_multi_tensor_adam": [I, I, P, P, I, F, F, F, F, F, F, F, I, P, P, P, P, P],
            "pha_multi_tensor_momentum": [I, I, P, P, I, F, F, F, I, P],
            "pha_multi_tensor_l2sq": [P, P, I, P, P, P],
            "pha_bn_num_blocks": [LG, I],
            "pha_bn_fwd_train": [I, P, P, P, LG, I, P, P, P, P, P, P, P, P, P, F, F, I, P, I, P],
            "pha_bn_apply": [I, P, P, P, LG, I, P, P, I, P],
            "pha_bn_bwd": [I, P, P, P, LG, I, P, P, P, P, P, P, P, P, P, I, P, P, I, P],
            "pha_chunk_size": [],
            "pha_tensor_meta_size": [],
        }
        for name, args in sig.items():
            f = getattr(L, name, None)
            if f is None:
                continue
            f.argtypes = args
            f.restype = c_int
        for name in ("pha_flash_attn_fwd", "pha_flash_attn_bwd", "pha_flash_attn_bwd_preprocess"):
            if hasattr(L, name):
                getattr(L, name).restype = c_int
        _sigs_done = True
    return L


def _stream(t):
    return c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _ptr(t):
    return None if t is None else c_void_p(t.data_ptr())


def _check(rc, name):
    if rc != 0:
        raise RuntimeError(f"{name} failed with hipError {rc}")


# ----------------------------------------------------------------------------
# layer norm / softmax
# ----------------------------------------------------------------------------
def layer_norm_fwd(x, w, b, eps, residual=None):
    """y = LN(x) — or, with ``residual``, hs = x + residual and y = LN(hs) in one pass.
    Returns (y, mean, rstd) or (y, mean, rstd, hs)."""
    H = w.numel()
    rows = x.numel() // H
    assert x.numel() == rows * H and H % 8 == 0 and H <= 4096
    y = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    hs = None
    if residual is not None:
        assert residual.shape == x.shape and residual.dtype == x.dtype and residual.is_contiguous()
        hs = torch.empty_like(x)
    _check(_L().pha_layer_norm_fwd2(_DT[x.dtype], _DT[w.dtype], _ptr(x), _ptr(residual), _ptr(hs), _ptr(w.contiguous()),
                                    _ptr(None if b is None else b.contiguous()), _ptr(y), _ptr(mean), _ptr(rstd), rows, H,
                                    float(eps), _stream(x)), "layer_norm_fwd")
    return (y, mean, rstd) if residual is None else (y, mean, rstd, hs)


def layer_norm_bwd(dy, x, w, mean, rstd, has_bias, dres=None, dx_colsum=None):
    """dx = LN'(dy) (+ dres: gradient of a fused residual sum). ``x`` is the normalised input.
    dx_colsum (a dtype: fp32 or x's): also return the column sums of dx in it — the gradient of a
    bias that was folded into the forward's residual sum (add_layer_norm's ``xb``)."""
    H = w.numel()
    rows = x.numel() // H
    nblocks = int(_L().pha_layer_norm_bwd_nblocks(rows, H))  # partials [nblocks, H]
    dx = torch.empty_like(x)
    dw = torch.empty_like(w)
    db = torch.empty_like(w) if has_bias else None
    if dres is not None:
        assert dres.shape == x.shape and dres.dtype == x.dtype and dres.is_contiguous()
    part = torch.empty((3 if dx_colsum else 2, nblocks + 8, H), dtype=torch.float32, device=x.device)  # + stage rows
    if dx_colsum is not None:
        xs_dt = dx_colsum if dx_colsum in (torch.float32, x.dtype) else torch.float32
        dxs = torch.empty(H, dtype=xs_dt, device=x.device)
        _check(_L().pha_layer_norm_bwd3(_DT[x.dtype], _DT[w.dtype], _DT[xs_dt], _ptr(dy), _ptr(x), _ptr(w), _ptr(mean), _ptr(rstd),
                                        _ptr(dres), _ptr(dx), _ptr(dw), _ptr(db), _ptr(dxs), _ptr(part[0]),
                                        _ptr(part[1]), _ptr(part[2]), nblocks, rows, H, _stream(x)), "layer_norm_bwd3")
        return dx, dw, db, dxs
    _check(_L().pha_layer_norm_bwd2(_DT[x.dtype], _DT[w.dtype], _ptr(dy), _ptr(x), _ptr(w), _ptr(mean), _ptr(rstd),
                                    _ptr(dres), _ptr(dx), _ptr(dw), _ptr(db), _ptr(part[0]), _ptr(part[1]), nblocks, rows, H,
                                    _stream(x)), "layer_norm_bwd")
    return dx, dw, db


def dropout_seed(device):
    """(host seed, device seed word or None) for a dropout site whose mask the backward regenerates.
    Eager: a fresh host seed. Inside a hipGraph capture the host value would be baked into every
    replay, so the kernels also xor in a device word: a per-device counter bumped by a captured
    kernel (each replay advances it) and copied for this site — the copy is what the site's
    backward reads, whatever later sites did to the counter."""
    seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
    buf = _SEED_BUFS.get(device)
    if buf is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("dropout inside a hipGraph capture needs one eager step first")
        buf = _SEED_BUFS[device] = torch.zeros(1, dtype=torch.int32, device=device)
    if not torch.cuda.is_current_stream_capturing():
        return seed, None
    out = torch.empty(1, dtype=torch.int32, device=device)
    L = _L()
    if hasattr(L, "pha_seed_bump"):   # ++counter and the site's copy in one captured kernel
        L.pha_seed_bump.argtypes = [c_void_p, c_void_p, c_void_p]
        L.pha_seed_bump.restype = c_int
        _check(L.pha_seed_bump(_ptr(buf), _ptr(out), _stream(buf)), "seed_bump")
        return seed, out
    buf.add_(1)
    return seed, buf.clone()


_SEED_BUFS = {}


def bdrln_fwd(x, xbias, residual, w, b, eps, seed, thresh, kscale, seed_dev=None):
    """fused_bias_dropout_residual_layer_norm forward: hs = residual + dropout(x + xbias), y = LN(hs).
    Returns (y, mean, rstd, hs)."""
    H = w.numel()
    rows = x.numel() // H
    assert x.numel() == rows * H and H % 8 == 0 and H <= 4096
    assert residual.shape == x.shape and residual.dtype == x.dtype and residual.is_contiguous() and x.is_contiguous()
    y, hs = torch.empty_like(x), torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    xb = None if xbias is None else xbias.contiguous()
    if xb is not None and xb.dtype not in (torch.float32, x.dtype):
        xb = xb.float()
    xbdt = _DT[w.dtype] if xb is None else _DT[xb.dtype]
    _check(_L().pha_bdrln_fwd2(_DT[x.dtype], _DT[w.dtype], xbdt, _ptr(x), _ptr(xb), _ptr(residual), _ptr(hs),
                              _ptr(w.contiguous()), _ptr(None if b is None else b.contiguous()), _ptr(y), _ptr(mean),
                              _ptr(rstd), rows, H, float(eps), int(seed), int(thresh), float(kscale), _stream(x),
                              _ptr(seed_dev)),
           "bdrln_fwd")
    return y, mean, rstd, hs


def layer_norm_dropout_bwd(dy, x, w, mean, rstd, has_bias, seed, thresh, kscale, seed_dev=None):
    """The bias-free fused_bias_dropout_residual_layer_norm backward in one pass: returns
    (dh, dx, dw, db) with dh = LN'(dy) (the residual's gradient) and dx = dh * mask * kscale (the
    forward's regenerated mask) — layer_norm_bwd + dropout_bias_bwd without re-reading dh."""
    H = w.numel()
    rows = x.numel() // H
    nblocks = int(_L().pha_layer_norm_bwd_nblocks(rows, H))
    dh, dx = torch.empty_like(x), torch.empty_like(x)
    dw = torch.empty_like(w)
    db = torch.empty_like(w) if has_bias else None
    part = torch.empty((2, nblocks + 8, H), dtype=torch.float32, device=x.device)
    _check(_L().pha_layer_norm_dropout_bwd(_DT[x.dtype], _DT[w.dtype], _ptr(dy), _ptr(x), _ptr(w), _ptr(mean),
                                           _ptr(rstd), _ptr(dh), _ptr(dx), _ptr(dw), _ptr(db), _ptr(part[0]),
                                           _ptr(part[1]), nblocks, rows, H, int(seed), int(thresh), float(kscale),
                                           _stream(x), _ptr(seed_dev)),
           "layer_norm_dropout_bwd")
    return dh, dx, dw, db


def dropout_bias_bwd(dh, seed, thresh, kscale, bias_dtype=None, seed_dev=None):
    """dx = dh * mask * kscale (the forward's regenerated mask) and dbias = column sums of dx."""
    H = dh.shape[-1]
    rows = dh.numel() // H
    nblocks = int(_L().pha_layer_norm_bwd_nblocks(rows, H))
    dx = torch.empty_like(dh)
    db = torch.empty(H, dtype=bias_dtype, device=dh.device) if bias_dtype is not None else None
    wdt = _DT[bias_dtype] if bias_dtype is not None else _DT[dh.dtype]
    part = torch.empty((nblocks + 8, H), dtype=torch.float32, device=dh.device)
    _check(_L().pha_dropout_bias_bwd(_DT[dh.dtype], wdt, _ptr(dh), _ptr(dx), _ptr(db), _ptr(part), nblocks, rows, H,
                                     int(seed), int(thresh), float(kscale), _stream(dh), _ptr(seed_dev)),
           "dropout_bias_bwd")
    return dx, db


# ----------------------------------------------------------------------------
# batch norm (channels-last [M, C] view), optional fused residual-add + ReLU
# ----------------------------------------------------------------------------
def bn_supported(x, C):
    return x.is_cuda and x.dtype in _DT and x.is_contiguous() and C % 8 == 0 and x.numel() > 0 and x.shape[-1] == C


def bn_fwd_train(x, w, b, running_mean, running_var, eps, momentum, residual=None, relu=False, ext_stats=None):
    """x: [..., C] contiguous (NHWC). Returns y, save_mean, save_istd. Updates running stats in place.
    ext_stats = (partials [rows][2][C] fp32, rows): unshifted channel sums / sums of squares of x
    already computed by x's producer (the conv epilogue) — the statistics pass over x is skipped."""
    C = x.shape[-1]
    M = x.numel() // C
    assert bn_supported(x, C) and w.dtype == torch.float32 and w.numel() == C
    assert residual is None or (residual.shape == x.shape and residual.dtype == x.dtype and residual.is_contiguous())
    assert running_mean is None or (running_mean.dtype == torch.float32 and running_mean.is_contiguous())
    L = _L()
    nb = L.pha_bn_num_blocks(M, C)
    f32 = dict(dtype=torch.float32, device=x.device)
    part = torch.empty((max(nb, 64) + 64) * 2 * C, **f32)
    stats = torch.empty(4, C, **f32)  # save_mean, save_istd, scale, shift
    y = torch.empty_like(x)
    _check(L.pha_bn_fwd_train(_DT[x.dtype], _ptr(x), _ptr(residual), _ptr(y), M, C, _ptr(w), _ptr(b),
                              _ptr(running_mean), _ptr(running_var), _ptr(stats[0]), _ptr(stats[1]), _ptr(stats[2]),
                              _ptr(stats[3]), _ptr(part), float(eps), float(momentum), int(relu),
                              _ptr(ext_stats[0]) if ext_stats else None, int(ext_stats[1]) if ext_stats else 0,
                              _stream(x)),
           "bn_fwd_train")
    return y, stats[0], stats[1], stats[2:4]


def bn_apply(x, scale, shift, residual=None, relu=False):
    C = x.shape[-1]
    M = x.numel() // C
    assert bn_supported(x, C) and scale.dtype == torch.float32 and scale.numel() == C and shift.numel() == C
    y = torch.empty_like(x)
    _check(_L().pha_bn_apply(_DT[x.dtype], _ptr(x), _ptr(residual), _ptr(y), M, C, _ptr(scale.contiguous()),
                             _ptr(shift.contiguous()), int(relu), _stream(x)), "bn_apply")
    return y


def bn_bwd(dy, x, y, w, save_mean, save_istd, relu=False, want_dres=False, affine=None, ext_part=None):
    """affine ([2, C] fp32 forward scale / shift): with relu and y None the ReLU mask is recomputed
    from x (no residual in the forward), so y need not be kept or read."""
    C = x.shape[-1]
    M = x.numel() // C
    assert bn_supported(x, C) and dy.shape == x.shape and dy.dtype == x.dtype and dy.is_contiguous()
    assert not relu or (y is not None and y.shape == x.shape) or (affine is not None and affine.shape == (2, C))
    L = _L()
    nb = L.pha_bn_num_blocks(M, C)
    f32 = dict(dtype=torch.float32, device=x.device)
    part = torch.empty((max(nb, 64) + 64) * 2 * C, **f32)
    coef = torch.empty(3 * C, **f32)
    dwb = torch.empty(2, C, **f32)
    dx = torch.empty_like(x)
    dres = torch.empty_like(x) if want_dres else None
    _check(L.pha_bn_bwd(_DT[x.dtype], _ptr(dy), _ptr(x), _ptr(y), M, C, _ptr(w), _ptr(save_mean), _ptr(save_istd),
                        _ptr(dx), _ptr(dres), _ptr(dwb[0]), _ptr(dwb[1]), _ptr(part), _ptr(coef), int(relu),
                        _ptr(affine.contiguous()) if affine is not None else None,
                        _ptr(ext_part[0]) if ext_part else None, int(ext_part[1]) if ext_part else 0, _stream(x)),
           "bn_bwd")
    return dx, dwb[0], dwb[1], dres


def softmax_fwd(x):
    H = x.shape[-1]
    rows = x.numel() // H
    assert H % 8 == 0 and H <= 4096
    y = torch.empty_like(x)
    _check(_L().pha_softmax_fwd(_DT[x.dtype], _ptr(x), _ptr(y), rows, H, _stream(x)), "softmax_fwd")
    return y


def softmax_bwd(dy, y):
    H = y.shape[-1]
    rows = y.numel() // H
    dx = torch.empty_like(y)
    _check(_L().pha_softmax_bwd(_DT[y.dtype], _ptr(dy), _ptr(y), _ptr(dx), rows, H, _stream(y)), "softmax_bwd")
    return dx


# ----------------------------------------------------------------------------
# cross entropy / gelu / embedding
# ----------------------------------------------------------------------------
def softmax_ce_fwd(logits, labels, ignore_index):
    rows, V = logits.shape
    assert labels.numel() == rows and V > 0   # V % 8 != 0: the kernels' element-wise path
    loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
    lse = torch.empty(rows, dtype=torch.float32, device=logits.device)
    _check(_L().pha_softmax_ce_fwd(_DT[logits.dtype], _ptr(logits), _ptr(labels), _ptr(loss), _ptr(lse), rows, V,
                                   int(ignore_index), _stream(logits)), "softmax_ce_fwd")
    return loss, lse


def softmax_ce_bwd(gloss, logits, labels, lse, ignore_index):
    rows, V = logits.shape
    dx = torch.empty_like(logits)
    _check(_L().pha_softmax_ce_bwd(_DT[logits.dtype], _ptr(gloss), _ptr(logits), _ptr(labels), _ptr(lse), _ptr(dx), rows, V,
                                   int(ignore_index), _stream(logits)), "softmax_ce_bwd")
    return dx


def bias_gelu_fwd(x, b, approximate):
    n = x.numel()
    H = x.shape[-1]
    if n % 8 or (b is not None and (H % 8 or b.numel() != H)):
        import torch.nn.functional as TF
        return TF.gelu(x + b if b is not None else x, approximate="tanh" if approximate else "none")
    y = torch.empty_like(x)
    _check(_L().pha_bias_gelu_fwd(_DT[x.dtype], _ptr(x), _ptr(b), _ptr(y), n, H, int(approximate), _stream(x)), "bias_gelu_fwd")
    return y


def bias_gelu_bwd(gy, x, b, approximate, want_db=True):
    """(d(gelu(x + b)) / dx . gy, its column sums — the bias gradient; None with want_db=False, for
    callers that take it from the next weight-gradient GEMM, ops/gemm.mm_tn_db)"""
    n = x.numel()
    H = x.shape[-1]
    if n % 8 or (b is not None and H % 8):
        xx = (x + b if b is not None else x).detach().float().requires_grad_(True)
        import torch.nn.functional as TF
        with torch.enable_grad():
            y = TF.gelu(xx, approximate="tanh" if approximate else "none")
            (gx,) = torch.autograd.grad(y, xx, gy.float())
        gx = gx.to(x.dtype)
    elif b is not None and not want_db and x.dtype != torch.float32:
        gx = torch.empty_like(x)
        rows = n // H
        rpb = max(16, -(-rows // 512))
        L = _L()
        L.pha_bias_gelu_bwd_rows.restype = c_int
        _check(L.pha_bias_gelu_bwd_rows(_DT[x.dtype], _ptr(gy), _ptr(x), _ptr(b), _ptr(gx), c_int(rows), c_int(H),
                                        c_int(rpb), c_int(int(approximate)), _stream(x)), "bias_gelu_bwd_rows")
        return gx, None
    elif b is not None and want_db and x.dtype != torch.float32 and hasattr(_L(), "pha_bias_gelu_bwd_db"):
        # gx and the per-row-block column sums of gx in one pass; db = sum of the partials
        gx = torch.empty_like(x)
        rows = n // H
        rpb = max(16, -(-rows // 512))   # >= 2048 blocks at 16384 x 8192: 8 per CU for streaming
        P = -(-rows // rpb)
        part = torch.empty((P + 8, H), dtype=torch.float32, device=x.device)   # + column-sum stage rows
        L = _L()
        L.pha_bias_gelu_bwd_db.restype = c_int
        _check(L.pha_bias_gelu_bwd_db(_DT[x.dtype], _ptr(gy), _ptr(x), _ptr(b), _ptr(gx), _ptr(part), c_int(rows),
                                      c_int(H), c_int(rpb), c_int(int(approximate)), _stream(x)), "bias_gelu_bwd_db")
        return gx, _col_sum_rows(part, P, b.dtype)
    else:
        gx = torch.empty_like(x)
        _check(_L().pha_bias_gelu_bwd(_DT[x.dtype], _ptr(gy), _ptr(x), _ptr(b), _ptr(gx), n, H, int(approximate), _stream(x)), "bias_gelu_bwd")
    gb = gx.reshape(-1, H).sum(0, dtype=torch.float32).to(b.dtype) if b is not None and want_db else None
    return gx, gb


def col_sum(gy2d, out_dtype=None):
    """column sums of a [rows, H] bf16/fp16 tensor (a linear layer's bias gradient): row-block
    partials in fp32 on the HIP kernel, then one small reduction of the partials"""
    rows, H = gy2d.shape
    if gy2d.dtype == torch.float32 or H % 8 or not gy2d.is_contiguous():
        return gy2d.sum(0, dtype=torch.float32).to(out_dtype or gy2d.dtype)
    rpb = max(16, -(-rows // 512))
    P = -(-rows // rpb)
    part = torch.empty((P + 8, H), dtype=torch.float32, device=gy2d.device)   # + column-sum stage rows
    L = _L()
    L.pha_col_sum_partial.restype = c_int
    _check(L.pha_col_sum_partial(_DT[gy2d.dtype], _ptr(gy2d), _ptr(part), c_int(rows), c_int(H), c_int(rpb),
                                 _stream(gy2d)), "col_sum_partial")
    return _col_sum_rows(part, P, out_dtype or gy2d.dtype)


def _col_sum_rows(part, P, dtype):
    """column sums of the first P rows of the fp32 partials ``part`` ([P + 8, H]: the last rows are
    the kernel's first-stage workspace) into a new [H] tensor of ``dtype``"""
    H = part.shape[1]
    if dtype not in _DT or not hasattr(_L(), "pha_col_sum_rows"):
        return part[:P].sum(0).to(dtype)
    out = torch.empty(H, dtype=dtype, device=part.device)
    _check(_L().pha_col_sum_rows(_DT[dtype], _ptr(part), _ptr(out), P, H, _stream(part)), "col_sum_rows")
    return out


class MaxPool2dNHWC(torch.autograd.Function):
    """NHWC max pool on the HIP kernels: forward keeps the window position of each max (1 byte per
    output element), backward gathers per input pixel (no atomics, no scatter)."""

    @staticmethod
    def forward(ctx, x, k, s, p):
        N, H, W, C = x.shape
        OH = (H + 2 * p[0] - k[0]) // s[0] + 1
        OW = (W + 2 * p[1] - k[1]) // s[1] + 1
        y = torch.empty(N, OH, OW, C, dtype=x.dtype, device=x.device)
        idx = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=x.device)
        L = _L()
        L.pha_maxpool2d_nhwc_fwd.restype = c_int
        _check(L.pha_maxpool2d_nhwc_fwd(_DT[x.dtype], _ptr(x), _ptr(y), _ptr(idx), *[c_int(v) for v in (
            N, H, W, C, OH, OW, k[0], k[1], s[0], s[1], p[0], p[1])], _stream(x)), "maxpool2d_nhwc_fwd")
        ctx.save_for_backward(idx)
        ctx.conf = (x.shape, k, s, p)
        return y

    @staticmethod
    def backward(ctx, gy):
        idx, = ctx.saved_tensors
        (N, H, W, C), k, s, p = ctx.conf
        gy = gy.contiguous()
        gx = torch.empty(N, H, W, C, dtype=gy.dtype, device=gy.device)
        L = _L()
        L.pha_maxpool2d_nhwc_bwd.restype = c_int
        _check(L.pha_maxpool2d_nhwc_bwd(_DT[gy.dtype], _ptr(gy), _ptr(idx), _ptr(gx), *[c_int(v) for v in (
            N, H, W, C, idx.shape[1], idx.shape[2], k[0], k[1], s[0], s[1], p[0], p[1])], _stream(gy)),
               "maxpool2d_nhwc_bwd")
        return gx, None, None, None


def maxpool_nhwc_ok(x, k, s, p):
    return (x.is_cuda and x.dim() == 4 and x.dtype in _DT and x.shape[-1] % 8 == 0 and x.is_contiguous()
            and k[0] * k[1] <= 256 and p[0] < k[0] and p[1] < k[1] and hasattr(_L(), "pha_maxpool2d_nhwc_fwd"))


def embedding_fwd(ids, w):
    ids = ids.to(torch.int64)
    rows = ids.numel()
    D = w.shape[1]
    out = torch.empty(list(ids.shape) + [D], dtype=w.dtype, device=w.device)
    if rows == 0:
        return out
    _check(_L().pha_embedding_fwd(_ptr(ids), _ptr(w), _ptr(out), rows, D * w.element_size(), w.shape[0], _stream(w)), "embedding_fwd")
    return out


def embedding_bwd(ids, gy, vocab, padding_idx=None):
    """dW [vocab, D] of an embedding lookup: deterministic (token-order sums, no atomics, no sort)"""
    ids = ids.reshape(-1).to(torch.int64).contiguous()
    D = gy.shape[-1]
    gy2 = gy.reshape(-1, D).contiguous()
    gw = torch.empty(vocab, D, dtype=gy.dtype, device=gy.device)
    pad = -1 if padding_idx is None else int(padding_idx) % vocab
    n = ids.numel()
    # a small vocabulary (token types, positions) gives few (row, column) blocks: split the tokens
    # into chunks (>= 1024 tokens each) so ~512 blocks stream them, fp32 partials summed in order
    blocks = -(-vocab // 32) * -(-D // 1024)
    chunks = 1
    if blocks < 512 and n >= 2048:
        chunks = max(1, min(-(-512 // blocks), n // 1024, 65535))
    ws = torch.empty(chunks, vocab, D, dtype=torch.float32, device=gy.device) if chunks > 1 else None
    _check(_L().pha_embedding_bwd(_DT[gy.dtype], _ptr(ids), _ptr(gy2), _ptr(gw), n, D, vocab, pad,
                                  _stream(gy), chunks, _ptr(ws)), "embedding_bwd")
    return gw


def embedding_bwd_supported(gy, n):
    return gy.dtype in _DT and gy.shape[-1] % 4 == 0 and n < (1 << 26) and n > 0


# ----------------------------------------------------------------------------
# multi-tensor optimizers
# ----------------------------------------------------------------------------
_META_DT = np.dtype([("p", "<u8"), ("g", "<u8"), ("m", "<u8"), ("v", "<u8"), ("master", "<u8"),
                     ("n", "<i8"), ("lr", "<f4"), ("wd", "<f4")])
_NORM_DT = np.dtype([("x", "<u8"), ("n", "<i8"), ("dt", "<i4"), ("pad", "<i4")])


def _chunk():
    return _L().pha_chunk_size()


class _CaptureStaging:
    """Page-locked host staging for pointer tables built while a hipGraph is being captured.
    torch's pinned caching allocator records an event on the capturing stream, which HIP refuses,
    so a table uploaded during capture is written into a block of this hipHostMalloc arena
    (allocated on the first eager upload, i.e. before any capture) and copied by a
    hipMemcpyAsync that the graph records as a memcpy node. Blocks are never reused: the graph
    re-reads them on every replay."""
    SIZE = 8 << 20

    def __init__(self):
        import ctypes
        self._ct = ctypes
        self._hip = ctypes.CDLL("libamdhip64.so")
        self._hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        self._hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                             ctypes.c_void_p]
        p = ctypes.c_void_p()
        rc = self._hip.hipHostMalloc(ctypes.byref(p), self.SIZE, 0)
        if rc != 0:
            raise RuntimeError(f"hipHostMalloc failed ({rc})")
        self._base, self._used = p.value, 0

    def upload(self, raw, device):
        n = raw.nbytes
        off = (self._used + 255) & ~255
        if off + n > self.SIZE:
            raise RuntimeError("hipGraph capture staging exhausted (pointer tables of too many captures)")
        self._used = off + n
        self._ct.memmove(self._base + off, raw.ctypes.data, n)
        dst = torch.empty(n, dtype=torch.uint8, device=device)
        rc = self._hip.hipMemcpyAsync(dst.data_ptr(), self._base + off, n, 1,
                                      torch.cuda.current_stream(device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"hipMemcpyAsync failed during capture ({rc})")
        return dst


_staging = None


def _upload(arr, device):
    global _staging
    raw = np.ascontiguousarray(arr.view(np.uint8))
    if torch.cuda.is_current_stream_capturing():
        if _staging is None:
            raise RuntimeError("pointer tables built during a hipGraph capture need one eager step first")
        return _staging.upload(raw, device)
    if _staging is None and torch.cuda.is_available():
        _staging = _CaptureStaging()
    host = torch.from_numpy(raw.copy()).pin_memory()
    return host.to(device, non_blocking=True)


def _group_by_dtype(items, key):
    groups = {}
    for it in items:
        groups.setdefault(key(it), []).append(it)
    return groups


class _TablePlan:
    """Cached (metas, chunks) device tables for a fixed list of tensors."""

    def __init__(self):
        self.key = None
        self.tables = None


_plans = {}


def _build_tables(recs, device, chunk):
    meta = np.zeros(len(recs), dtype=_META_DT)
    chunks = []
    for i, r in enumerate(recs):
        meta[i] = r
        n = int(r[5])
        for c in range((n + chunk - 1) // chunk):
            chunks.append((i, c))
    ch = np.asarray(chunks, dtype=np.int32).reshape(-1, 2)
    return _upload(meta, device), _upload(ch, device), len(chunks)


def _tables_cached(tag, recs, device):
    """Pointer tables are rebuilt only when any pointer/size changes (steady state: cached)."""
    key = tuple(tuple(r[:6]) + (r[6], r[7]) for r in recs)
    plan = _plans.get(tag)
    if plan is not None and plan[0] == key:
        return plan[1]
    t = _build_tables(recs, device, _chunk())
    _plans[tag] = (key, t)
    return t


def multi_tensor_adam(params, grads, ms, vs, masters, lr, beta1, beta2, eps, step, weight_decay, decoupled,
                      lr_ratios, grad_scale, wds=None, gscale_dev=None, lr_dev=None, pow_dev=None):
    """gscale_dev: optional fp32 device scalar multiplied into every gradient as it is read (the
    global-norm clip factor — no separate pass over the gradients). lr_dev / pow_dev: fp32 device
    scalars (learning rate; (beta1^t, beta2^t) before this update) read by the kernel instead of
    the host values — what a hipGraph-captured step needs so that replays advance."""
    L = _L()
    dev = params[0].device
    items = []
    for i, p in enumerate(params):
        g = grads[i]
        if g is None:
            continue
        mst = masters[i] if masters is not None else None
        wd = wds[i] if wds is not None else weight_decay
        rec = (p.data_ptr(), g.data_ptr(), ms[i].data_ptr(), vs[i].data_ptr(), 0 if mst is None else mst.data_ptr(),
               p.numel(), float(lr_ratios[i]) if lr_ratios is not None else 1.0, float(wd))
        items.append((p.dtype, g.dtype, rec))
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    stream = _stream(params[0])
    for (pdt, gdt), its in _group_by_dtype(items, lambda t: (t[0], t[1])).items():
        metas, chunks, n = _tables_cached(("adam", pdt, gdt), [t[2] for t in its], dev)
        _check(L.pha_multi_tensor_adam(_DT[pdt], _DT[gdt], _ptr(metas), _ptr(chunks), n, float(lr), float(beta1), float(beta2),
                                       float(eps), float(bc1), float(bc2), float(grad_scale), int(bool(decoupled)),
                                       _ptr(gscale_dev), _ptr(lr_dev), _ptr(None if pow_dev is None else pow_dev[0]),
                                       _ptr(None if pow_dev is None else pow_dev[1]), stream),
               "multi_tensor_adam")
    _bump([p for p, g in zip(params, grads) if g is not None])


def multi_tensor_momentum(params, grads, vels, masters, lr, mu, nesterov, weight_decay, lr_ratios, grad_scale, wds=None):
    L = _L()
    dev = params[0].device
    items = []
    for i, p in enumerate(params):
        g = grads[i]
        if g is None:
            continue
        mst = masters[i] if masters is not None else None
        wd = wds[i] if wds is not None else weight_decay
        rec = (p.data_ptr(), g.data_ptr(), vels[i].data_ptr(), 0, 0 if mst is None else mst.data_ptr(), p.numel(),
               float(lr_ratios[i]) if lr_ratios is not None else 1.0, float(wd))
        items.append((p.dtype, g.dtype, rec))
    stream = _stream(params[0])
    for (pdt, gdt), its in _group_by_dtype(items, lambda t: (t[0], t[1])).items():
        metas, chunks, n = _tables_cached(("mom", pdt, gdt), [t[2] for t in its], dev)
        _check(L.pha_multi_tensor_momentum(_DT[pdt], _DT[gdt], _ptr(metas), _ptr(chunks), n, float(lr), float(mu),
                                           float(grad_scale), int(bool(nesterov)), stream), "multi_tensor_momentum")
    _bump([p for p, g in zip(params, grads) if g is not None])


def _bump(params):
    """The multi-tensor kernels write parameters through raw pointers, invisible to torch's
    version counters: bump them, so version-keyed caches of derived layouts (conv filter
    re-layouts, transposed linear weights) and autograd's saved-tensor checks see the update."""
    if params:
        torch.autograd.graph.increment_version(params)


def multi_tensor_l2norm_sq(tensors):
    L = _L()
    dev = tensors[0].device
    chunk = _chunk()
    meta = np.zeros(len(tensors), dtype=_NORM_DT)
    chunks = []
    for i, t in enumerate(tensors):
        assert t.is_contiguous()
        meta[i] = (t.data_ptr(), t.numel(), _DT[t.dtype], 0)
        for c in range((t.numel() + chunk - 1) // chunk):
            chunks.append((i, c))
    ch = np.asarray(chunks, dtype=np.int32).reshape(-1, 2)
    out = torch.empty(1, dtype=torch.float32, device=dev)
    partial = torch.empty(max(1, len(chunks)), dtype=torch.float32, device=dev)
    meta_d = _upload(meta, dev)   # keep the device tables alive until the launch is enqueued
    ch_d = _upload(ch, dev)
    _check(L.pha_multi_tensor_l2sq(_ptr(meta_d), _ptr(ch_d), len(chunks), _ptr(partial), _ptr(out), _stream(tensors[0])),
           "multi_tensor_l2sq")
    # the caching allocator may hand these blocks out again once freed; tie them to the stream
    meta_d.record_stream(torch.cuda.current_stream(dev))
    ch_d.record_stream(torch.cuda.current_stream(dev))
    return out[0]


# ----------------------------------------------------------------------------
# flash attention (csrc/kernels/flash_attn.hip)
# ----------------------------------------------------------------------------
def flash_attn_supported(q, k, v, dropout_p, mask=None):
    """shapes the own kernels take: bf16/fp16 [B, S, H, D] with D <= 256 (32 / 64 / 128 / 256
    natively, other multiples of 8 zero-padded up; 256 on the generic 4-wave kernels), GQA (H % Hk == 0); optional additive / boolean mask
    broadcastable to [B, H, S, Sk] that needs no gradient; optional dropout"""
    import os
    if os.environ.get("PHA_DISABLE_FLASH") == "1":
        return False
    L = _lib.lib
    if L is None or not hasattr(L, "pha_flash_attn_fwd"):
        return False
    if q.dtype not in (torch.bfloat16, torch.float16) or k.dtype != q.dtype or v.dtype != q.dtype:
        return False
    if q.dim() != 4 or k.dim() != 4 or v.dim() != 4:
        return False
    B, S, H, D = q.shape
    if D > 256 or D % 8 or k.shape != v.shape or k.shape[0] != B or k.shape[3] != D:
        return False
    if D > 128 and os.environ.get("PHA_FA_WIDE", "sdpa") != "own":
        # head dims 129-256 run on the generic 4-wave kernels at one wave per SIMD (the backward
        # spills): correct and tested, but 2.5x slower than torch SDPA at D = 256
        # (profiles/fa_d256_r3.log) — opt in with PHA_FA_WIDE=own
        return False
    if H % k.shape[2] != 0:
        return False
    if dropout_p and not (0.0 < dropout_p < 1.0):
        return False
    if mask is not None:
        if not isinstance(mask, torch.Tensor) or mask.requires_grad or mask.dim() > 4:
            return False
        try:
            torch.broadcast_shapes(tuple(mask.shape), (B, H, S, k.shape[1]))
        except RuntimeError:
            return False
    return True


def _fa_head_dim(D):
    return D if D in (32, 64, 128, 256) else (64 if D < 64 else 128 if D < 128 else 256)


def _fa_bias(mask, B, H, S, Sk, device):
    """additive fp32 bias view [B, H, S, Sk] (broadcast dims stride 0, keys contiguous) and its
    (batch, head, query) element strides"""
    if mask.dtype == torch.bool:
        mask = torch.zeros(mask.shape, dtype=torch.float32, device=device).masked_fill_(~mask.to(device), float("-inf"))
    else:
        mask = mask.to(device=device, dtype=torch.float32)
    while mask.dim() < 4:
        mask = mask.unsqueeze(0)
    if mask.stride(-1) != 1 and mask.shape[-1] != 1:
        mask = mask.contiguous()
    if mask.shape[-1] == 1:   # broadcast over keys: materialise the key dimension
        mask = mask.expand(*mask.shape[:-1], Sk).contiguous()
    mask = mask.expand(B, H, S, Sk)
    return mask, (mask.stride(0), mask.stride(1), mask.stride(2))


def _fa64_on(D, mask, Sk=None):
    """head dim 64: the 8-wave LDS-DMA kernels of flash_attn_d64.hip (packed strides, in-kernel
    dropout whose keep bits the forward stores for the backward, an additive mask read as float4 key
    quads: Sk % 4 == 0); PHA_FA64=0 keeps the generic 4-wave kernels"""
    import os
    L = _lib.lib
    return (D == 64 and (mask is None or (Sk is not None and Sk % 4 == 0)) and L is not None
            and hasattr(L, "pha_fa64_fwd") and os.environ.get("PHA_FA64", "1") != "0")


def _fa64_bias(mask, B, H, S, Sk, device):
    """(bias view, (sb, sh, sq)) for the D = 64 kernels, or (None, (0, 0, 0))"""
    if mask is None:
        return None, (0, 0, 0)
    bias, st = _fa_bias(mask, B, H, S, Sk, device)
    if bias.data_ptr() % 16 or any(x % 4 for x in st):
        bias = bias.contiguous()
        st = (bias.stride(0), bias.stride(1), bias.stride(2))
    return bias, st


def _fa64_sig(L):
    if not getattr(L, "_fa64_sig", False):
        P, I, LG, F, U = c_void_p, c_int, c_long, c_float, ctypes.c_uint
        L.pha_fa64_fwd.argtypes = [I, P, P, P, P, P, I, I, I, I, I, F, I, LG, I, LG, I, LG, I, F, U, P, P, P,
                                   P, LG, LG, LG]
        L.pha_fa64_fwd.restype = c_int
        L.pha_fa64_bwd.argtypes = [I, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, I, LG, I, LG, I, LG, I, LG, I,
                                   LG, I, F, U, P, P, P, P, LG, LG, LG]
        L.pha_fa64_mask_words.argtypes = [I]
        L.pha_fa64_mask_words.restype = c_int
        L.pha_fa64_mask_size.argtypes = [I, I, I, I]
        L.pha_fa64_mask_size.restype = c_long
        L.pha_fa64_bwd.restype = c_int
        L._fa64_sig = True
    return L


def _fa64_fwd(dt, qp, kp, vp, o, lse, B, S, Sk, H, Hk, sc, causal, qs, kvs, os_, dropout_p, seed, seed_dev, st,
              bias=None, bst=(0, 0, 0)):
    """qs / kvs / os_: (token, head) element strides of q, k / v and o. With dropout, returns the keep
    mask as bits (int32 [B * H][words][S up to 64]) for the backward — the reference fused attention keeps
    its dropout mask too (fmha_ref.h dropout_mask_out); PHA_FA64_MASKBITS=0 re-hashes instead"""
    import os
    L = _fa64_sig(_L())
    dmask = None
    if dropout_p and os.environ.get("PHA_FA64_MASKBITS", "1") != "0":
        dmask = torch.empty(L.pha_fa64_mask_size(B, H, S, Sk), dtype=torch.int32, device=o.device)
    _check(L.pha_fa64_fwd(dt, qp, kp, vp, _ptr(o), _ptr(lse), B, S, Sk, H, Hk, sc, int(causal), qs[0], qs[1], kvs[0],
                          kvs[1], os_[0], os_[1], float(dropout_p), seed, _ptr(seed_dev), st, _ptr(dmask),
                          _ptr(bias), bst[0], bst[1], bst[2]),
           "fa64_fwd")
    return dmask


def _fa64_bwd(dt, qp, kp, vp, do, lse, delta, dqp, dkp, dvp, B, S, Sk, H, Hk, sc, causal, qs, kvs, gqs, gkvs,
              dropout_p, seed, seed_dev, st, dmask=None, bias=None, bst=(0, 0, 0)):
    L = _fa64_sig(_L())
    _check(L.pha_fa64_bwd(dt, qp, kp, vp, _ptr(do), _ptr(lse), _ptr(delta), dqp, dkp, dvp, B, S, Sk, H, Hk, sc,
                          int(causal), qs[0], qs[1], kvs[0], kvs[1], H * 64, 64, gqs[0], gqs[1], gkvs[0], gkvs[1],
                          float(dropout_p), seed, _ptr(seed_dev), st, _ptr(dmask), _ptr(bias), bst[0], bst[1],
                          bst[2]), "fa64_bwd")


class FlashAttentionExt(torch.autograd.Function):
    """Flash attention with an additive mask and / or dropout (4-wave kernels, head dims
    32 / 64 / 128): the dropout mask is a counter-based hash of (seed, b*H+h, query, key),
    regenerated in the backward instead of stored."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale, mask, dropout_p):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        B, S, H, D = q.shape
        Sk, Hk = k.shape[1], k.shape[2]
        sc = float(scale) if scale is not None else 1.0 / float(np.sqrt(D))
        bias, (sb, sh, sq) = (None, (0, 0, 0)) if mask is None else _fa_bias(mask, B, H, S, Sk, q.device)
        seed, seed_dev = dropout_seed(q.device) if dropout_p else (0, None)
        o = torch.empty_like(q)
        lse = torch.empty((B, H, S), dtype=torch.float32, device=q.device)
        ctx.fa64 = _fa64_on(D, mask, Sk)
        if ctx.fa64:
            b64, bst = _fa64_bias(mask, B, H, S, Sk, q.device)
            ctx.dmask = _fa64_fwd(_DT[q.dtype], _ptr(q), _ptr(k), _ptr(v), o, lse, B, S, Sk, H, Hk, sc, causal,
                                  (H * D, D), (Hk * D, D), (H * D, D), dropout_p, seed, seed_dev, _stream(q),
                                  b64, bst)
            ctx.save_for_backward(q, k, v, o, lse)
            ctx.bias, ctx.strides, ctx.seed, ctx.seed_dev = b64, bst, seed, seed_dev
            ctx.causal, ctx.scale, ctx.dropout_p = causal, sc, float(dropout_p)
            return o
        L = _L()
        if not getattr(L, "_fa_ext_sig", False):
            P, I, LG, F, U = c_void_p, c_int, c_long, c_float, ctypes.c_uint
            L.pha_flash_attn_fwd_ext.argtypes = [I, P, P, P, P, P, I, I, I, I, I, I, F, I, P, LG, LG, LG, F, U, P, P]
            L.pha_flash_attn_fwd_ext.restype = c_int
            L.pha_flash_attn_bwd_ext.argtypes = [I, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, F, I, P, LG, LG, LG,
                                                 F, U, P, LG, I, LG, I, P]
            L.pha_flash_attn_bwd_ext.restype = c_int
            L._fa_ext_sig = True
        _check(L.pha_flash_attn_fwd_ext(_DT[q.dtype], _ptr(q), _ptr(k), _ptr(v), _ptr(o), _ptr(lse), B, S, Sk, H, Hk, D,
                                        sc, int(causal), _ptr(bias), sb, sh, sq, float(dropout_p), seed, _stream(q),
                                        _ptr(seed_dev)),
               "flash_attn_fwd_ext")
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.bias, ctx.strides, ctx.seed, ctx.seed_dev = bias, (sb, sh, sq), seed, seed_dev
        ctx.causal, ctx.scale, ctx.dropout_p = causal, sc, float(dropout_p)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        do = do.contiguous()
        B, S, H, D = q.shape
        Sk, Hk = k.shape[1], k.shape[2]
        L = _L()
        delta = torch.empty((B, H, S), dtype=torch.float32, device=q.device)
        dq = torch.empty_like(q)
        dk = torch.empty_like(k) if Hk == H else torch.empty((B, Sk, H, D), dtype=k.dtype, device=k.device)
        dv = torch.empty_like(v) if Hk == H else torch.empty((B, Sk, H, D), dtype=v.dtype, device=v.device)
        _check(L.pha_flash_attn_bwd_preprocess(c_int(_DT[q.dtype]), _ptr(o), _ptr(do), _ptr(delta), c_int(B), c_int(S),
                                               c_int(H), c_int(D), _stream(q)), "flash_attn_bwd_preprocess")
        if getattr(ctx, "fa64", False):
            _fa64_bwd(_DT[q.dtype], _ptr(q), _ptr(k), _ptr(v), do, lse, delta, _ptr(dq), _ptr(dk), _ptr(dv), B, S, Sk,
                      H, Hk, ctx.scale, ctx.causal, (H * D, D), (Hk * D, D), (0, 0), (0, 0), ctx.dropout_p, ctx.seed,
                      ctx.seed_dev, _stream(q), ctx.dmask, ctx.bias, ctx.strides)
        else:
            sb, sh, sq = ctx.strides
            _check(L.pha_flash_attn_bwd_ext(_DT[q.dtype], _ptr(q), _ptr(k), _ptr(v), _ptr(do), _ptr(lse), _ptr(delta),
                                            _ptr(dq), _ptr(dk), _ptr(dv), B, S, Sk, H, Hk, D, ctx.scale,
                                            int(ctx.causal), _ptr(ctx.bias), sb, sh, sq, ctx.dropout_p, ctx.seed,
                                            _stream(q), 0, 0, 0, 0, _ptr(ctx.seed_dev)),
                   "flash_attn_bwd_ext")
        if Hk != H:
            g = H // Hk
            dk = dk.view(B, Sk, Hk, g, D).sum(3)
            dv = dv.view(B, Sk, Hk, g, D).sum(3)
        return dq, dk, dv, None, None, None, None


class FlashAttentionExtPacked(torch.autograd.Function):
    """FlashAttentionExt on a packed [B, S, H, 3D] projection (q | k | v per head, the BERT / fused
    QKV layout): the forward takes dense copies of the three slices, the backward writes dq / dk /
    dv straight into ONE packed [B, S, H, 3D] gradient through the kernels' output strides — no
    concatenation pass (0.67 ms per BERT-base step, profiles/README.md round 5)"""

    @staticmethod
    def forward(ctx, qkv, causal, scale, mask, dropout_p):
        B, S, H, D3 = qkv.shape
        D = D3 // 3
        ctx.fa64p = _fa64_on(D, mask, S) and qkv.is_contiguous()
        if ctx.fa64p:   # head dim 64: the kernels read q | k | v in place (no slice copies)
            sc = float(scale) if scale is not None else 1.0 / float(np.sqrt(D))
            seed, seed_dev = dropout_seed(qkv.device) if dropout_p else (0, None)
            o = torch.empty((B, S, H, D), dtype=qkv.dtype, device=qkv.device)
            lse = torch.empty((B, H, S), dtype=torch.float32, device=qkv.device)
            es, base = qkv.element_size(), qkv.data_ptr()
            b64, bst = _fa64_bias(mask, B, H, S, S, qkv.device)
            ctx.dmask = _fa64_fwd(_DT[qkv.dtype], c_void_p(base), c_void_p(base + D * es),
                                  c_void_p(base + 2 * D * es), o, lse, B, S, S, H, H, sc, causal, (3 * H * D, 3 * D),
                                  (3 * H * D, 3 * D), (H * D, D), dropout_p, seed, seed_dev, _stream(qkv), b64, bst)
            ctx.b64, ctx.bst = b64, bst
            ctx.save_for_backward(qkv, o, lse)
            ctx.seed, ctx.seed_dev, ctx.causal, ctx.scale, ctx.dropout_p = seed, seed_dev, causal, sc, float(dropout_p)
            return o
        q, k, v = (qkv[..., i * D:(i + 1) * D].contiguous() for i in range(3))
        o = FlashAttentionExt.forward(ctx, q, k, v, causal, scale, mask, dropout_p)
        return o

    @staticmethod
    def backward(ctx, do):
        if ctx.fa64p:
            qkv, o, lse = ctx.saved_tensors
            do = do.contiguous()
            B, S, H, D3 = qkv.shape
            D = D3 // 3
            L = _L()
            delta = torch.empty((B, H, S), dtype=torch.float32, device=qkv.device)
            g = torch.empty_like(qkv)
            _check(L.pha_flash_attn_bwd_preprocess(c_int(_DT[qkv.dtype]), _ptr(o), _ptr(do), _ptr(delta), c_int(B),
                                                   c_int(S), c_int(H), c_int(D), _stream(qkv)),
                   "flash_attn_bwd_preprocess")
            es, base, gb = qkv.element_size(), qkv.data_ptr(), g.data_ptr()
            st = (3 * H * D, 3 * D)
            _fa64_bwd(_DT[qkv.dtype], c_void_p(base), c_void_p(base + D * es), c_void_p(base + 2 * D * es), do, lse,
                      delta, c_void_p(gb), c_void_p(gb + D * es), c_void_p(gb + 2 * D * es), B, S, S, H, H, ctx.scale,
                      ctx.causal, st, st, st, st, ctx.dropout_p, ctx.seed, ctx.seed_dev, _stream(qkv), ctx.dmask,
                      ctx.b64, ctx.bst)
            return g, None, None, None, None
        q, k, v, o, lse = ctx.saved_tensors
        do = do.contiguous()
        B, S, H, D = q.shape
        L = _L()
        delta = torch.empty((B, H, S), dtype=torch.float32, device=q.device)
        g = torch.empty((B, S, H, 3 * D), dtype=q.dtype, device=q.device)
        _check(L.pha_flash_attn_bwd_preprocess(c_int(_DT[q.dtype]), _ptr(o), _ptr(do), _ptr(delta), c_int(B), c_int(S),
                                               c_int(H), c_int(D), _stream(q)), "flash_attn_bwd_preprocess")
        sb, sh, sq = ctx.strides
        es = g.element_size()
        base = g.data_ptr()
        _check(L.pha_flash_attn_bwd_ext(_DT[q.dtype], _ptr(q), _ptr(k), _ptr(v), _ptr(do), _ptr(lse), _ptr(delta),
                                        c_void_p(base), c_void_p(base + D * es), c_void_p(base + 2 * D * es), B, S, S,
                                        H, H, D, ctx.scale, int(ctx.causal), _ptr(ctx.bias), sb, sh, sq, ctx.dropout_p,
                                        ctx.seed, _stream(q), 3 * H * D, 3 * D, 3 * H * D, 3 * D, _ptr(ctx.seed_dev)),
               "flash_attn_bwd_ext(packed)")
        return g, None, None, None, None


def flash_attention_packed_ext(qkv, causal, scale, mask=None, dropout_p=0.0):
    """attention over a packed [B, S, H, 3D] projection with a mask and / or dropout (head dims 32 /
    64 / 128 / 256); None when the ext kernels cannot take it (the caller splits instead)"""
    B, S, H, D3 = qkv.shape
    D = D3 // 3
    if D3 % 3 or D not in (32, 64, 128, 256) or not qkv.is_cuda or qkv.dtype not in (torch.bfloat16, torch.float16):
        return None
    q = qkv[..., :D]
    if not flash_attn_supported(q, q, q, dropout_p, mask):
        return None
    sc = float(scale) if scale is not None else 1.0 / float(np.sqrt(D))
    return FlashAttentionExtPacked.apply(qkv, bool(causal), sc, mask, float(dropout_p))


def flash_attention_any(q, k, v, causal, scale, mask=None, dropout_p=0.0):
    """dispatch: the 8-wave D=128 / 4-wave D=64 kernels without mask or dropout, the extension
    kernels otherwise; head dims other than 32 / 64 / 128 are zero-padded up"""
    D = q.shape[-1]
    Dp = _fa_head_dim(D)
    sc = float(scale) if scale is not None else 1.0 / float(np.sqrt(D))
    if Dp != D:
        pad = (0, Dp - D)
        q, k, v = (torch.nn.functional.pad(t, pad) for t in (q, k, v))
    if mask is None and not dropout_p and Dp in (64, 128):
        o = FlashAttention.apply(q, k, v, bool(causal), sc)
    else:
        o = FlashAttentionExt.apply(q, k, v, bool(causal), sc, mask, float(dropout_p or 0.0))
    return o[..., :D] if Dp != D else o


def _bwd_fused(D):
    """Single-kernel backward (dK, dV and atomically summed dQ) when PHA_FA_BWD=fused; the default
    is the two-kernel v2 backward, measured faster at the GPT shape (0.95 vs 1.14 ms, B8 S2048
    H16 D128 causal: the fused kernel's one wave per SIMD exposes its LDS latency)."""
    import os
    if D != 128 or os.environ.get("PHA_FA_BWD", "v2") != "fused" or os.environ.get("PHA_FA_BWD_V1") == "1":
        return False
    return hasattr(_lib.lib, "pha_flash_attn_bwd_fused")


class FlashAttention(torch.autograd.Function):
    """Forward/backward on our MFMA flash-attention kernels. Layout [B, S, H, D]."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        B, S, H, D = q.shape
        Sk, Hk = k.shape[1], k.shape[2]
        sc = float(scale) if scale is not None else 1.0 / float(np.sqrt(D))
        o = torch.empty_like(q)
        lse = torch.empty((B, H, S), dtype=torch.float32, device=q.device)
        ctx.fa64 = _fa64_on(D, None)
        if ctx.fa64:
            _fa64_fwd(_DT[q.dtype], _ptr(q), _ptr(k), _ptr(v), o, lse, B, S, Sk, H, Hk, sc, causal, (H * D, D),
                      (Hk * D, D), (H * D, D), 0.0, 0, None, _stream(q))
        else:
            L = _L()
            _check(L.pha_flash_attn_fwd(c_int(_DT[q.dtype]), _ptr(q), _ptr(k), _ptr(v), _ptr(o), _ptr(lse), c_int(B),
                                        c_int(S), c_int(Sk), c_int(H), c_int(Hk), c_int(D), c_float(sc),
                                        c_int(int(causal)), _stream(q)), "flash_attn_fwd")
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal = causal
        ctx.scale = sc
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        do = do.contiguous()
        B, S, H, D = q.shape
        Sk, Hk = k.shape[1], k.shape[2]
        L = _L()
        delta = torch.empty((B, H, S), dtype=torch.float32, device=q.device)
        dq = torch.empty_like(q)
        dk = torch.empty_like(k) if Hk == H else torch.empty((B, Sk, H, D), dtype=k.dtype, device=k.device)
        dv = torch.empty_like(v) if Hk == H else torch.empty((B, Sk, H, D), dtype=v.dtype, device=v.device)
        _check(L.pha_flash_attn_bwd_preprocess(c_int(_DT[q.dtype]), _ptr(o), _ptr(do), _ptr(delta), c_int(B), c_int(S), c_int(H), c_int(D),
                                               _stream(q)), "flash_attn_bwd_preprocess")
        if getattr(ctx, "fa64", False):
            _fa64_bwd(_DT[q.dtype], _ptr(q), _ptr(k), _ptr(v), do, lse, delta, _ptr(dq), _ptr(dk), _ptr(dv), B, S, Sk,
                      H, Hk, ctx.scale, ctx.causal, (H * D, D), (Hk * D, D), (0, 0), (0, 0), 0.0, 0, None, _stream(q))
        elif _bwd_fused(D):
            # single-kernel backward; dQ is summed over key blocks in an fp32 workspace
            acc = torch.empty((B, S, H, D), dtype=torch.float32, device=q.device)
            L.pha_flash_attn_bwd_fused.restype = c_int
            _check(L.pha_flash_attn_bwd_fused(c_int(_DT[q.dtype]), _ptr(q), _ptr(k), _ptr(v), _ptr(do), _ptr(lse),
                                              _ptr(delta), _ptr(dq), _ptr(dk), _ptr(dv), _ptr(acc), c_int(B), c_int(S),
                                              c_int(Sk), c_int(H), c_int(Hk), c_int(D), c_float(ctx.scale),
                                              c_int(int(ctx.causal)), _stream(q)), "flash_attn_bwd_fused")
        else:
            _check(L.pha_flash_attn_bwd(c_int(_DT[q.dtype]), _ptr(q), _ptr(k), _ptr(v), _ptr(do), _ptr(lse), _ptr(delta), _ptr(dq),
                                        _ptr(dk), _ptr(dv), c_int(B), c_int(S), c_int(Sk), c_int(H), c_int(Hk), c_int(D),
                                        c_float(ctx.scale), c_int(int(ctx.causal)), _stream(q)), "flash_attn_bwd")
        if Hk != H:
            g = H // Hk
            dk = dk.view(B, Sk, Hk, g, D).sum(3)
            dv = dv.view(B, Sk, Hk, g, D).sum(3)
        return dq, dk, dv, None, None


def flash_attn_packed_supported(qkv, num_heads):
    """qkv: [B, S, H, 3D] contiguous projection output (q|k|v per head), D == 128."""
    import os
    if os.environ.get("PHA_DISABLE_FLASH") == "1" or os.environ.get("PHA_FA_FWD_V1") == "1" \
            or os.environ.get("PHA_FA_BWD_V1") == "1":
        return False
    L = _lib.lib
    return (L is not None and hasattr(L, "pha_flash_attn_fwd_packed") and qkv.is_cuda and qkv.dim() == 4
            and qkv.dtype in (torch.bfloat16, torch.float16) and qkv.is_contiguous() and qkv.shape[2] == num_heads
            and qkv.shape[3] == 3 * 128)


class FlashAttentionPacked(torch.autograd.Function):
    """Self-attention straight from the fused QKV projection [B, S, H, 3D]: the kernels read q/k/v
    in place (strided) and the backward writes dq/dk/dv into one packed [B, S, H, 3D] gradient,
    so neither the three split copies nor the concat of their gradients exists."""

    @staticmethod
    def forward(ctx, qkv, causal, scale):
        B, S, H, D3 = qkv.shape
        D = D3 // 3
        sc = float(scale) if scale is not None else 1.0 / float(np.sqrt(D))
        o = torch.empty((B, S, H, D), dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty((B, H, S), dtype=torch.float32, device=qkv.device)
        L = _L()
        L.pha_flash_attn_fwd_packed.restype = c_int
        _check(L.pha_flash_attn_fwd_packed(c_int(_DT[qkv.dtype]), _ptr(qkv), _ptr(o), _ptr(lse), c_int(B), c_int(S),
                                           c_int(H), c_int(D), c_float(sc), c_int(int(causal)), _stream(qkv)),
               "flash_attn_fwd_packed")
        ctx.save_for_backward(qkv, o, lse)
        ctx.causal, ctx.scale = causal, sc
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        do = do.contiguous()
        B, S, H, D3 = qkv.shape
        D = D3 // 3
        L = _L()
        L.pha_flash_attn_bwd_packed.restype = c_int
        delta = torch.empty((B, H, S), dtype=torch.float32, device=qkv.device)
        dqkv = torch.empty_like(qkv)
        if not _bwd_fused(D) and hasattr(L, "pha_flash_attn_bwd_packed_od"):
            # delta = rowsum(dO * O) formed inside the dQ kernel (no separate preprocess pass)
            L.pha_flash_attn_bwd_packed_od.restype = c_int
            _check(L.pha_flash_attn_bwd_packed_od(c_int(_DT[qkv.dtype]), _ptr(qkv), _ptr(o), _ptr(do), _ptr(lse),
                                                  _ptr(delta), _ptr(dqkv), c_int(B), c_int(S), c_int(H), c_int(D),
                                                  c_float(ctx.scale), c_int(int(ctx.causal)), _stream(qkv)),
                   "flash_attn_bwd_packed_od")
            return dqkv, None, None
        _check(L.pha_flash_attn_bwd_preprocess(c_int(_DT[qkv.dtype]), _ptr(o), _ptr(do), _ptr(delta), c_int(B),
                                               c_int(S), c_int(H), c_int(D), _stream(qkv)), "flash_attn_bwd_preprocess")
        if _bwd_fused(D):
            acc = torch.empty((B, S, H, D), dtype=torch.float32, device=qkv.device)
            L.pha_flash_attn_bwd_packed_fused.restype = c_int
            _check(L.pha_flash_attn_bwd_packed_fused(c_int(_DT[qkv.dtype]), _ptr(qkv), _ptr(do), _ptr(lse),
                                                     _ptr(delta), _ptr(dqkv), _ptr(acc), c_int(B), c_int(S), c_int(H),
                                                     c_int(D), c_float(ctx.scale), c_int(int(ctx.causal)),
                                                     _stream(qkv)), "flash_attn_bwd_packed_fused")
        else:
            _check(L.pha_flash_attn_bwd_packed(c_int(_DT[qkv.dtype]), _ptr(qkv), _ptr(do), _ptr(lse), _ptr(delta),
                                               _ptr(dqkv), c_int(B), c_int(S), c_int(H), c_int(D), c_float(ctx.scale),
                                               c_int(int(ctx.causal)), _stream(qkv)), "flash_attn_bwd_packed")
        return dqkv, None, None
